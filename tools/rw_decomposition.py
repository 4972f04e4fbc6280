#!/usr/bin/env python3
"""Where do the mix's bytes go? The 8-neighbour mix (9 reads + 1 write of P fp32) against its
two halves on the same buffers: the 9 reads alone (mode 3) and the output write alone (mode 4),
grid-stride like the production kernel, several occupancies. Interleaved rounds, one process.
GB/s uses each variant's own algorithmic bytes (mix 10 P * 4, reads 9 P * 4, write P * 4).
By default (round 3) the stacks are placement-calibrated (federated_amd.placement.calibrated_stacks,
as the bench's) and the production mix (cfa_mix_seq_f32, its default shape) runs beside the
variants; --plain: one plain allocation per stack (round 1's profiles/r01_rw_decomposition.jsonl)."""
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
fn = lib.cfa_experimental_mix8_traverse
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_float),
               ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
al = _lib.float_array([1.0 / 9] * 8)
PLACED = "--plain" not in sys.argv
if PLACED:
    from federated_amd.placement import calibrated_stacks
    m, o, report = calibrated_stacks(L, P, torch.device("cuda", 0), eng, 4, 4, candidates=4, rows=L)
    m.normal_()
    print(json.dumps({"placement": {k: report[k] for k in ("chosen", "plain_us", "chosen_us") if k in report}}),
          flush=True)
else:
    m = torch.empty(L, P, device="cuda").normal_()
    o = torch.empty(L, P, device="cuda")
st = torch.cuda.current_stream().cuda_stream
variants = [("mix", 0, 2, 10), ("reads_only", 3, 2, 9), ("write_only", 4, 2, 1),
            ("mix_bpc4", 0, 4, 10), ("reads_only_bpc4", 3, 4, 9), ("write_only_bpc4", 4, 4, 1),
            ("reads_only_bpc1", 3, 1, 9), ("write_only_bpc8", 4, 8, 1)]
if PLACED:
    variants = [("production", None, None, 10), ("mix_bpc1", 0, 1, 10)] + variants + [("write_only_bpc1", 4, 1, 1)]
alphas = [1.0 / 9] * 8


def run(v):
    for k in range(MIXES):
        i = k % L
        nb = [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)]
        if v[1] is None:
            eng.mix_seq(o[i], m[i], nb, alphas)
            continue
        rc = fn(o[i].data_ptr(), m[i].data_ptr(), _lib.ptr_table([x.data_ptr() for x in nb]), al, P, v[1], v[2], st)
        assert rc == 0, lib.cfa_exp_last_error()


times = {v[0]: [] for v in variants}
for _ in range(R):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(v)
        e1.record()
        torch.cuda.synchronize()
        times[v[0]].append(e0.elapsed_time(e1) / MIXES)
for v in variants:
    med = statistics.median(times[v[0]])
    print(json.dumps({"variant": v[0], "blocks_per_cu": v[2], "us": round(med * 1e3, 2),
                      "GBps": round(v[3] * P * 4 / (med * 1e-3) / 1e9, 1)}), flush=True)
