#!/usr/bin/env python3
"""Store form of the streaming mix at the production launch shape (one workgroup per CU, two float4
per lane): the production global nt loads with the output stored through a buffer store sc1
(production), a global store nt, a buffer store nt, a global store sc1 or sc1 nt
(cfa_experimental_mix8_store), n = 8, P = 25M, on placement-calibrated ring stacks as the bench's.
Interleaved rounds, one process; every variant's output equals production bit for bit.
GPU box: python tools/probe/store_form.py"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.placement import calibrated_stacks  # noqa: E402

P, L, R, MIXES = 25_000_000, 16, 4, 32
eng = get_engine(0)
lib = _lib.load_experiments()
fn = lib.cfa_experimental_mix8_store
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_float),
               ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
alphas = [1.0 / 9] * 8
al = _lib.float_array(alphas)
m, o, report = calibrated_stacks(L, P, torch.device("cuda", 0), eng, 4, 4, candidates=4, rows=L)
m.normal_()
print(json.dumps({"placement": {k: report[k] for k in ("chosen", "plain_us", "chosen_us")}}), flush=True)
st = torch.cuda.current_stream().cuda_stream
# (name, u, store mode, blocks per CU); u None = production
variants = [("production", None, None, None), ("buffer_sc1", 2, 0, 1), ("global_nt", 2, 1, 1),
            ("buffer_nt", 2, 2, 1), ("global_sc1", 2, 3, 1), ("global_sc1_nt", 2, 4, 1),
            ("global_nt_u1", 1, 1, 1), ("global_nt_u4", 4, 1, 1)]
if os.environ.get("STORE_SHAPES"):  # nt store at other launch shapes (workgroups per CU x float4 per lane)
    variants = [("production", None, None, None), ("global_nt", 2, 1, 1), ("global_nt_b2", 2, 1, 2),
                ("global_nt_u1_b2", 1, 1, 2), ("global_nt_u4_b2", 4, 1, 2), ("global_nt_b3", 2, 1, 3),
                ("global_nt_u1_b4", 1, 1, 4), ("global_nt_u1_b3", 1, 1, 3), ("buffer_sc1_b2", 2, 0, 2)]


def nbrs(i):
    return [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)]


def mix(v, i):
    if v[1] is None:
        eng.mix_seq(o[i], m[i], nbrs(i), alphas)
        return
    rc = fn(o[i].data_ptr(), m[i].data_ptr(), _lib.ptr_table([x.data_ptr() for x in nbrs(i)]), al, P,
            v[1], v[2], v[3], st)
    assert rc == 0, lib.cfa_exp_last_error()


ref = torch.empty(P, device="cuda")
eng.mix_seq(ref, m[3], nbrs(3), alphas)
for v in variants:
    o[3].zero_()
    mix(v, 3)
    torch.cuda.synchronize()
    assert torch.equal(o[3], ref), v
print(json.dumps({"check": "every variant equals production bit for bit"}), flush=True)

times = {v[0]: [] for v in variants}
for _ in range(R):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(MIXES):
            mix(v, k % L)
        e1.record()
        torch.cuda.synchronize()
        times[v[0]].append(e0.elapsed_time(e1) / MIXES * 1e3)
for v in variants:
    med = statistics.median(times[v[0]])
    print(json.dumps({"variant": v[0], "vec_per_lane": v[1], "store_mode": v[2],
                      "blocks_per_cu": v[3], "us": round(med, 2), "min_us": round(min(times[v[0]]), 2),
                      "frac": round(10 * P * 4 / (med * 1e-6) / 1e9 / 8000, 4)}), flush=True)
