#!/usr/bin/env python3
"""Cache-policy sweep for the streaming mix (8 neighbours x P fp32): the experiment kernel
cfa_experimental_mix8_buf with explicit load/store aux bits (1 = sc0, 2 = nt, 16 = sc1),
interleaved rounds in one process, plus the production kernel as the reference row."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P, K, ROUNDS, LAUNCH = 25_001_984, 8, 5, 8  # P multiple of 4096
eng = get_engine(0)
lib = _lib.load_experiments()
fn = lib.cfa_experimental_mix8_buf
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_float),
               ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
sets = []
for _ in range(3):
    xs = [torch.randn(P, device="cuda") for _ in range(K + 1)]
    sets.append((xs[0], xs[1:], torch.empty(P, device="cuda")))
alphas = [1.0 / (K + 1)] * K
pairs = [(0, 0), (2, 2), (2, 0), (0, 2), (1, 2), (16, 2), (17, 2), (3, 2), (18, 2), (19, 2), (2, 16), (2, 17),
         (2, 18), (2, 19), (18, 18), (17, 17), (16, 16), (1, 1)]
pairs = [(2, 2), (2, 16), (2, 17)] + [(-2, s) for s in (0, 2, 16, 17, 18, 1)]
cfgs = [("buf" if l >= 0 else "gld+bst", l, s, b) for (l, s) in pairs for b in (2,)] + [("prod", -1, -1, 2)]
ref = torch.empty(P, device="cuda")
eng.mix_seq(ref, sets[0][0], sets[0][1], alphas)
st = torch.cuda.current_stream().cuda_stream


def launch(c, s):
    loc, nb, out = s
    if c[0] == "prod":
        eng.mix_seq(out, loc, nb, alphas)
    else:
        rc = fn(out.data_ptr(), loc.data_ptr(), _lib.ptr_table([x.data_ptr() for x in nb]), _lib.float_array(alphas),
                P, c[1], c[2], c[3], st)
        assert rc == 0, lib.cfa_exp_last_error()


times = {c: [] for c in cfgs}
for r in range(ROUNDS):
    for c in cfgs:
        if r == 0:
            launch(c, sets[0])
            torch.cuda.synchronize()
            assert torch.equal(sets[0][2], ref), c
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(LAUNCH):
            launch(c, sets[i % 3])
        e1.record()
        torch.cuda.synchronize()
        times[c].append(e0.elapsed_time(e1) / LAUNCH)
rows = []
for c, ts in times.items():
    med = statistics.median(ts)
    rows.append({"kernel": c[0], "load_aux": c[1], "store_aux": c[2], "blocks_per_cu": c[3],
                 "us": round(med * 1e3, 2), "GBps": round((K + 2) * P * 4 / (med * 1e-3) / 1e9, 1)})
for r in sorted(rows, key=lambda x: x["us"]):
    print(json.dumps(r))
