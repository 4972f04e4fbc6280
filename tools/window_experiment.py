#!/usr/bin/env python3
"""Same box, same process: is a sliding 9-row window over a stacked population (the bench's
round) slower per mix than rotating disjoint bucket sets (the tuning sweeps)? Interleaved."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

P, L, R = 25_000_000, 64, 4
eng = get_engine(0)
a = [1.0 / 9] * 8
stack = torch.empty(L, P, device="cuda").normal_()
out = torch.empty(L, P, device="cuda")
sets = [([torch.randn(P, device="cuda") for _ in range(9)], torch.empty(P, device="cuda")) for _ in range(3)]
perm = torch.randperm(L).tolist()


def sliding():
    for i in range(L):
        nb = [stack[(i + o) % L] for o in (-4, -3, -2, -1, 1, 2, 3, 4)]
        eng.mix_seq(out[i], stack[i], nb, a)


def scattered():  # stacked, but each mix's 9 rows far apart (stride 7 rows)
    for i in range(L):
        nb = [stack[(i + 7 * o) % L] for o in (-4, -3, -2, -1, 1, 2, 3, 4)]
        eng.mix_seq(out[i], stack[i], nb, a)


def rotating():
    for i in range(L):
        xs, o = sets[i % 3]
        eng.mix_seq(o, xs[0], xs[1:], a)


variants = {"sliding_window": sliding, "scattered_rows": scattered, "rotating_3_sets": rotating}
times = {k: [] for k in variants}
for _ in range(R):
    for k, f in variants.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / L)
for k, ts in times.items():
    m = statistics.median(ts)
    print(json.dumps({"variant": k, "us_per_mix": round(m * 1e3, 2), "GBps": round(1e9 / (m * 1e-3) / 1e9, 1)}))
