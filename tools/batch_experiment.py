#!/usr/bin/env python3
"""Write batching for the 8-neighbour mix (tools/rw_decomposition.py: the 9 reads alone run at
7.0 TB/s and the write alone at 5.5 TB/s, but interleaved the mix takes 18 us more than the two
apart). Each wave folds B tiles into LDS and then stores them in one burst; 'soft' also lines the
chip's bursts up with a bounded-spin arrival counter. Outputs are checked bit-equal to the
production kernel. Interleaved rounds on sliding windows of a 16-row stack, one process."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P, L, R, MIXES = 25_001_984, 16, 5, 32
eng = get_engine(0)
lib = _lib.load_experiments()
fn = lib.cfa_experimental_mix8_batch
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_float),
               ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
alphas = [1.0 / 9] * 8
al = _lib.float_array(alphas)
m = torch.empty(L, P, device="cuda").normal_()
o = torch.empty(L, P, device="cuda")
st = torch.cuda.current_stream().cuda_stream
spin = int(os.environ.get("SPIN", "400"))
variants = [("prod", None), ("batch1", (1, 0)), ("batch2", (2, 0)), ("batch4", (4, 0)),
            ("batch2_soft", (2, 1)), ("batch4_soft", (4, 1))]


def nbrs(i):
    return [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)]


def mix(v, i):
    if v[1] is None:
        eng.mix_seq(o[i], m[i], nbrs(i), alphas)
    else:
        b, soft = v[1]
        rc = fn(o[i].data_ptr(), m[i].data_ptr(), _lib.ptr_table([x.data_ptr() for x in nbrs(i)]), al, P, b, soft,
                spin, 2, st)
        assert rc == 0, lib.cfa_exp_last_error()


ref = torch.empty(P, device="cuda")
eng.mix_seq(ref, m[5], nbrs(5), alphas)
for v in variants:
    o[5].zero_()
    mix(v, 5)
    torch.cuda.synchronize()
    assert torch.equal(o[5], ref), v[0]
times = {v[0]: [] for v in variants}
for _ in range(R):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(MIXES):
            mix(v, k % L)
        e1.record()
        torch.cuda.synchronize()
        times[v[0]].append(e0.elapsed_time(e1) / MIXES)
for v in variants:
    med = statistics.median(times[v[0]])
    print(json.dumps({"variant": v[0], "spin_limit": spin, "us": round(med * 1e3, 2), "min_us": round(min(times[v[0]]) * 1e3, 2),
                      "GBps": round(10 * P * 4 / (med * 1e-3) / 1e9, 1)}), flush=True)
