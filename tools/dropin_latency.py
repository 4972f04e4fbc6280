#!/usr/bin/env python3
"""Per-call latency breakdown of the drop-in host path at the TF1 C1 shapes (2NN, P = 16 680,
2 neighbours): HostMixer.mix_tf1 (fp64 buckets), HostMixer.mix (fp32), the bare kernel on
device-resident buckets, and a plain H2D + D2H of the same bytes. Medians over 200 calls."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from federated_amd.consensus._runtime import mixer  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

rng = np.random.default_rng(0)
shapes = [(512, 32), (32,), (32, 8), (8,)]
local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(2)]
alphas = [0.5, 0.5]
mx = mixer()
eng = get_engine(0)
P = sum(int(np.prod(s)) for s in shapes)


def med(fn, n=200):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


d = [torch.randn(P, device="cuda") for _ in range(3)]
out = torch.empty(P, device="cuda")
h = torch.empty(3 * P, pin_memory=True)
dd = torch.empty(3 * P, device="cuda")
ho = torch.empty(P, pin_memory=True)


def kernel_only():
    eng.mix_seq(out, d[0], d[1:], alphas)
    torch.cuda.synchronize()


def copies_only():
    dd.copy_(h, non_blocking=True)
    ho.copy_(out, non_blocking=True)
    torch.cuda.synchronize()


from federated_amd.consensus import _runtime as R  # noqa: E402

R.SINGLE_ZERO_COPY = R.TF1_ZERO_COPY = False
t_copies = med(lambda: mx.mix(local, nbrs, alphas))
t_tf1_copies = med(lambda: mx.mix_tf1(local, nbrs, alphas))
R.SINGLE_ZERO_COPY = R.TF1_ZERO_COPY = True
res = {"P": P, "mix_tf1_us": med(lambda: mx.mix_tf1(local, nbrs, alphas)), "mix_tf1_staged_copies_us": t_tf1_copies,
       "mix_fp32_us": med(lambda: mx.mix(local, nbrs, alphas)), "mix_fp32_staged_copies_us": t_copies,
       "kernel_plus_sync_us": med(kernel_only), "h2d_d2h_plus_sync_us": med(copies_only),
       "sync_only_us": med(torch.cuda.synchronize)}
print(json.dumps(res))
