#!/usr/bin/env python3
"""Per-mix time of the sliding-window round against the touched footprint (L rows in, L rows
out, 100 MB each), everything allocated up front, interleaved in one process. Tests whether
the rotating-set advantage (3 GB touched vs 12.8 GB, tools/window_experiment.py) is a
footprint (address-translation reach) effect."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

P, R, MIXES = 25_000_000, 4, 64
eng = get_engine(0)
a = [1.0 / 9] * 8
Ls = [9, 16, 24, 32, 48, 64, 128]
pops = {L: (torch.empty(L, P, device="cuda").normal_(), torch.empty(L, P, device="cuda")) for L in Ls}


def run(L):
    m, o = pops[L]
    for k in range(MIXES):
        i = k % L
        eng.mix_seq(o[i], m[i], [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)], a)


times = {L: [] for L in Ls}
for _ in range(R):
    for L in Ls:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(L)
        e1.record()
        torch.cuda.synchronize()
        times[L].append(e0.elapsed_time(e1) / MIXES)
for L in Ls:
    m = statistics.median(times[L])
    print(json.dumps({"rows": L, "touched_GB": round(2 * L * P * 4 / 1e9, 1), "us_per_mix": round(m * 1e3, 2),
                      "GBps": round(1e9 / (m * 1e-3) / 1e9, 1)}))
