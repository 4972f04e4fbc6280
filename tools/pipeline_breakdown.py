#!/usr/bin/env python3
"""Where does HostMixer's chunked pipeline spend its time at 8 x 25M? Times (a) the whole
HostMixer.mix, (b) packing every chunk into pinned staging (no GPU), (c) the chunked H2D
copies alone (data already packed), (d) the unpack of the 100 MB result, (e) pack interleaved
with the async H2D of the previous chunk (the pipeline without kernels and D2H)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from federated_amd.consensus import _runtime as R  # noqa: E402
from federated_amd.engine import BucketLayout  # noqa: E402

K = 8
shapes = [(5000, 4000), (4000,), (1000, 4996), (4,)]
rng = np.random.default_rng(0)
models = [[rng.standard_normal(s, dtype=np.float32) for s in shapes] for _ in range(K + 1)]
lay = BucketLayout.of(models[0])
P = lay.P
mx = R.mixer()
al = [1.0 / (K + 1)] * K
C = 8
step = -(-P // C)
step += (-step) % 4
bounds = [(a, min(a + step, P)) for a in range(0, P, step)]
pad = lambda m: m + (-m) % 4
offs, total = [], 0
for a, b in bounds:
    offs.append(total)
    total += (K + 1) * pad(b - a)
host = torch.empty(total, dtype=torch.float32, pin_memory=True)
dev = torch.empty(total, dtype=torch.float32, device="cuda")
flat = [[torch.from_numpy(t.reshape(-1)) for t in m] for m in models]
seg = [lay.segment(k) for k in range(len(shapes))]
h2d = torch.cuda.Stream()


def pack_chunk(c):
    (a, b), o = bounds[c], offs[c]
    w = pad(b - a)
    for j in range(K + 1):
        for k, (lo, hi) in enumerate(seg):
            x, y = max(a, lo), min(b, hi)
            if x < y:
                host[o + j * w + x - a:o + j * w + y - a].copy_(flat[j][k][x - lo:y - lo])


def h2d_chunk(c):
    (a, b), o = bounds[c], offs[c]
    w = pad(b - a)
    with torch.cuda.stream(h2d):
        dev[o:o + (K + 1) * w].copy_(host[o:o + (K + 1) * w], non_blocking=True)


def med(fn, n=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e3, 2)


h_out = torch.empty(P, pin_memory=True)


def unpack():
    for k, shp in enumerate(shapes):
        lo, hi = seg[k]
        o = np.empty(shp, dtype=np.float32)
        torch.from_numpy(o.reshape(-1)).copy_(h_out[lo:hi])


def overlapped():
    for c in range(C):
        pack_chunk(c)
        h2d_chunk(c)


def is_pinned_view():
    return bool(host[offs[1]:offs[2]].is_pinned())


print(json.dumps({"hostmixer_mix_ms": med(lambda: mx.mix(models[0], models[1:], al)),
                  "pack_all_chunks_ms": med(lambda: [pack_chunk(c) for c in range(C)]),
                  "h2d_all_chunks_ms": med(lambda: [h2d_chunk(c) for c in range(C)]),
                  "unpack_ms": med(unpack), "pack_plus_async_h2d_ms": med(overlapped),
                  "staging_view_pinned": is_pinned_view()}))
