#!/usr/bin/env python3
"""Traversal order of the streaming mix vs physical placement. Several stacked populations are
allocated (each lands on different physical memory); on each, a sliding-window round runs with
traversal modes 0 = grid-stride (production order), 1 = blocked, 2 = XCD-grouped grid-stride,
plus the production kernel. Interleaved rounds, one process. Output must equal production."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P, L, R, STACKS, MIXES = 25_001_984, 16, 4, 5, 32
eng = get_engine(0)
lib = _lib.load_experiments()
fn = lib.cfa_experimental_mix8_traverse
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_float),
               ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
alphas = [1.0 / 9] * 8
al = _lib.float_array(alphas)
stacks = [(torch.empty(L, P, device="cuda").normal_(), torch.empty(L, P, device="cuda")) for _ in range(STACKS)]
st = torch.cuda.current_stream().cuda_stream
variants = [("prod", None, 2), ("grid_stride", 0, 2), ("blocked", 1, 2), ("xcd_grouped", 2, 2),
            ("blocked_bpc4", 1, 4), ("blocked_bpc1", 1, 1)]


def nbrs(m, i):
    return [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)]


def mix(v, m, o, i):
    if v[1] is None:
        eng.mix_seq(o[i], m[i], nbrs(m, i), alphas)
    else:
        rc = fn(o[i].data_ptr(), m[i].data_ptr(), _lib.ptr_table([x.data_ptr() for x in nbrs(m, i)]), al, P, v[1], v[2], st)
        assert rc == 0, lib.cfa_exp_last_error()


m0, o0 = stacks[0]
ref = torch.empty(P, device="cuda")
eng.mix_seq(ref, m0[3], nbrs(m0, 3), alphas)
for v in variants:
    o0[3].zero_()
    mix(v, m0, o0, 3)
    torch.cuda.synchronize()
    assert torch.equal(o0[3], ref), v

times = {(v[0], s): [] for v in variants for s in range(STACKS)}
for _ in range(R):
    for s, (m, o) in enumerate(stacks):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for k in range(MIXES):
                mix(v, m, o, k % L)
            e1.record()
            torch.cuda.synchronize()
            times[(v[0], s)].append(e0.elapsed_time(e1) / MIXES)
for v in variants:
    row = {"variant": v[0], "blocks_per_cu": v[2]}
    meds = [statistics.median(times[(v[0], s)]) * 1e3 for s in range(STACKS)]
    row["us_per_mix_by_stack"] = [round(x, 1) for x in meds]
    row["mean_us"] = round(sum(meds) / len(meds), 2)
    row["GBps_mean"] = round((10 * P * 4) / (row["mean_us"] * 1e-6) / 1e9, 1)
    print(json.dumps(row), flush=True)
