#!/usr/bin/env python3
"""Software-pipelined streaming mix (cfa_experimental_mix_pipe, tools/experiments/cfa_experiments.hip)
against the production kernels, n = 8, P = 25M, on the same buffers: the loads of a workgroup's
next tile are issued before the current tile is folded and stored. Sequential rule (against
cfa_mix_seq_f32, the headline) and the FedAvg divisor fold (against cfa_mix_seq_div_f32).
Several stacked ring populations (each lands on its own physical memory), interleaved rounds,
one process. Outputs must equal production bit for bit. GPU box: python tools/probe/pipe_mix.py"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P = int(os.environ.get("PIPE_P", 25_000_000))
L, R, STACKS, MIXES = 16, int(os.environ.get("PIPE_ROUNDS", 4)), int(os.environ.get("PIPE_STACKS", 3)), 32
eng = get_engine(0)
lib = _lib.load_experiments()
fn = lib.cfa_experimental_mix_pipe
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_float),
               ctypes.POINTER(ctypes.c_float), ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
               ctypes.c_void_p]
alphas = [1.0 / 9] * 8
divs = [9.0] * 8
ones = [1.0] * 8
al, dv, on = _lib.float_array(alphas), _lib.float_array(divs), _lib.float_array(ones)
stacks = [(torch.empty(L, P, device="cuda").normal_(), torch.empty(L, P, device="cuda")) for _ in range(STACKS)]
st = torch.cuda.current_stream().cuda_stream
# (name, rule, u, blocks_per_cu); u None = production entry point
if os.environ.get("PIPE_NT"):  # round 3 follow-up: the divisor fold with a nontemporal store
    VARIANTS_NT = [("prod_seq", 0, None, None), ("pipe_seq_u2_b1_nt", 10, 2, 1), ("prod_div", 2, None, None),
                   ("pipe_div_u2_b1", 2, 2, 1), ("pipe_div_u2_b1_nt", 12, 2, 1), ("pipe_div_u1_b1_nt", 12, 1, 1),
                   ("pipe_div_u2_b2_nt", 12, 2, 2), ("pipe_div_u1_b2_nt", 12, 1, 2)]
variants = [("prod_seq", 0, None, None), ("pipe_seq_u1_b1", 0, 1, 1), ("pipe_seq_u2_b1", 0, 2, 1),
            ("pipe_seq_u4_b1", 0, 4, 1), ("pipe_seq_u1_b2", 0, 1, 2), ("pipe_seq_u2_b2", 0, 2, 2),
            ("prod_div", 2, None, None), ("pipe_div_u1_b1", 2, 1, 1), ("pipe_div_u1_b2", 2, 1, 2),
            ("pipe_div_u2_b1", 2, 2, 1), ("pipe_div_u2_b2", 2, 2, 2)]
if os.environ.get("PIPE_NT"):
    variants = VARIANTS_NT


def nbrs(m, i):
    return [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)]


def mix(v, m, o, i):
    name, rule, u, bpc = v
    base_rule = rule % 10
    if u is None:
        if base_rule == 0:
            eng.mix_seq(o[i], m[i], nbrs(m, i), alphas)
        else:
            eng.mix_seq_div(o[i], m[i], nbrs(m, i), ones, divs)
        return
    coeff = al if base_rule == 0 else on
    rc = fn(o[i].data_ptr(), m[i].data_ptr(), _lib.ptr_table([x.data_ptr() for x in nbrs(m, i)]), coeff,
            dv if base_rule == 2 else None, P, rule, u, bpc, st)
    assert rc == 0, lib.cfa_exp_last_error()


m0, o0 = stacks[0]
refs = {}
for rule in (0, 2):
    refs[rule] = torch.empty(P, device="cuda")
    if rule == 0:
        eng.mix_seq(refs[rule], m0[3], nbrs(m0, 3), alphas)
    else:
        eng.mix_seq_div(refs[rule], m0[3], nbrs(m0, 3), ones, divs)
for v in variants:
    o0[3].zero_()
    mix(v, m0, o0, 3)
    torch.cuda.synchronize()
    assert torch.equal(o0[3], refs[v[1] % 10]), v
print(json.dumps({"check": "every variant equals its production kernel bit for bit", "P": P}), flush=True)

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
    row = {"variant": v[0], "rule": v[1], "vec_per_lane": v[2], "blocks_per_cu": v[3]}
    meds = [statistics.median(times[(v[0], s)]) * 1e3 for s in range(STACKS)]
    row["us_per_mix_by_stack"] = [round(x, 1) for x in meds]
    row["mean_us"] = round(sum(meds) / len(meds), 2)
    row["GBps_mean"] = round((10 * P * 4) / (row["mean_us"] * 1e-6) / 1e9, 1)
    row["frac"] = round(row["GBps_mean"] / 8000, 4)
    print(json.dumps(row), flush=True)
