#!/usr/bin/env python3
"""One launch per device vs one launch per run of devices (cfa_experimental_mix8_multi) for a
ring population round at the bench shape (K = 8, 25M-class rows). Several stacks (each lands on
different physical memory), interleaved rounds, one process; outputs must be identical."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P = int(os.environ.get("MULTI_P", 25_001_984))  # MULTI_P=3125000 MULTI_L=128: one N = 8 params rank
L = int(os.environ.get("MULTI_L", 32))
R, STACKS = 4, 3
eng = get_engine(0)
lib = _lib.load_experiments()
fn = lib.cfa_experimental_mix8_multi
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
               ctypes.POINTER(ctypes.c_float), ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
alphas = [1.0 / 9] * 8
al = _lib.float_array(alphas)
st = torch.cuda.current_stream().cuda_stream
stacks = [(torch.empty(L, P, device="cuda").normal_(), torch.empty(L, P, device="cuda")) for _ in range(STACKS)]


def nbrs(m, i):
    return [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)]


def per_device(m, o):
    for i in range(L):
        eng.mix_seq(o[i], m[i], nbrs(m, i), alphas)


def multi(m, o, bpc=2):
    rc = fn(o.data_ptr(), m.data_ptr(), P, L, 0, L, al, P, bpc, st)
    assert rc == 0, lib.cfa_exp_last_error()


m0, o0 = stacks[0]
ref = torch.empty_like(o0)
per_device(m0, ref)
multi(m0, o0)
torch.cuda.synchronize()
assert torch.equal(o0, ref), "multi-device launch differs from per-device mixes"
del ref

variants = [("per_device", per_device), ("multi_bpc2", multi), ("multi_bpc4", lambda m, o: multi(m, o, 4))]
times = {(v, s): [] for v, _ in variants for s in range(STACKS)}
for _ in range(R):
    for s, (m, o) in enumerate(stacks):
        for name, f in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f(m, o)
            e1.record()
            torch.cuda.synchronize()
            times[(name, s)].append(e0.elapsed_time(e1) * 1e3 / L)
gb = 10 * P * 4 / 1e9
for (name, s), ts in times.items():
    us = statistics.median(ts)
    print(json.dumps({"experiment": "multi_mix", "variant": name, "stack": s, "devices": L, "P": P,
                      "us_per_device_mix": round(us, 2), "GBps": round(gb / (us * 1e-6), 1)}), flush=True)
