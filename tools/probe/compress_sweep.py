#!/usr/bin/env python3
"""Standalone compression epilogue (in place on y, DPCM reference read): variants of the tile
width, load / store policy and workgroups per CU against the production entry, 25M fp32,
interleaved rounds; counts checked equal."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P = 25_000_000
eng = get_engine(0)
exp = _lib.load_experiments()
fn = exp.cfa_experimental_compress
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
               ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
g = torch.Generator(device="cuda").manual_seed(1)
ref = torch.randn(P, device="cuda", generator=g) * 1e-3
y0 = ref + torch.randn(P, device="cuda", generator=g) * 1e-4
y = torch.empty_like(y0)
kept = eng.counter()
st = torch.cuda.current_stream().cuda_stream
cfgs = [("prod", 0, 0, 0, 0)] + [("x", u, l, s, b) for (u, l, s) in [(1, 1, 1), (2, 1, 1), (4, 1, 1), (8, 1, 1), (4, 1, 0),
                                                                       (4, 0, 1), (4, 0, 0), (2, 1, 0), (8, 1, 0)]
                                  for b in (2, 4)]


def launch(c):
    if c[0] == "prod":
        eng.compress(y, ref, 2, kept)
    else:
        assert fn(y.data_ptr(), ref.data_ptr(), P, 2, kept.data_ptr(), c[1], c[2], c[3], c[4], st) == 0


counts = {}
for c in cfgs:
    y.copy_(y0)
    kept.zero_()
    launch(c)
    torch.cuda.synchronize()
    counts[c] = int(kept.item())
assert len(set(counts.values())) == 1, counts
times = {c: [] for c in cfgs}
for _ in range(5):
    for c in cfgs:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            launch(c)
        b.record()
        torch.cuda.synchronize()
        times[c].append(a.elapsed_time(b) / 10)
for c in cfgs:
    ms = statistics.median(times[c])
    print(json.dumps({"variant": c[0], "U": c[1], "nt_load": c[2], "nt_store": c[3], "blocks_per_cu": c[4],
                      "us": round(ms * 1e3, 2), "frac": round(3 * P * 4 / (ms * 1e-3) / 8e12, 4)}))
