#!/usr/bin/env python3
"""Launch-shape sweep of the CFA mix kernel (K neighbours x P fp32) in ONE process with
interleaved rounds (cdna_hip_programming.md §5.4 rule 24). Prints a JSON line per config
with the median / min per-launch time and GB/s (algorithmic bytes (K+2)*P*4)."""
import argparse
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--neighbours", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--buffers", type=int, default=4, help="distinct input sets rotated (defeat MALL)")
    args = ap.parse_args()
    eng = get_engine(0)
    P, K = args.params, args.neighbours
    sets = []
    for b in range(args.buffers):
        xs = [torch.randn(P, device="cuda") for _ in range(K + 1)]
        sets.append((xs[0], xs[1:], torch.empty(P, device="cuda")))
    alphas = [1.0 / (K + 1)] * K
    cfgs = list(itertools.product([0, 1, 2, 3, 4, 8], [0, 1, 2, 4], [0, 1]))
    times = {c: [] for c in cfgs}
    ref = torch.empty(P, device="cuda")
    eng.mix_seq(ref, sets[0][0], sets[0][1], alphas)
    for r in range(args.rounds):
        for c in cfgs:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.launches)]
            for i, (a, b) in enumerate(evs):
                loc, nb, out = sets[i % len(sets)]
                a.record()
                eng.mix_seq(out, loc, nb, alphas, launch=c)
                b.record()
            torch.cuda.synchronize()
            times[c].extend(a.elapsed_time(b) for a, b in evs)
            if r == 0:
                eng.mix_seq(sets[0][2], sets[0][0], sets[0][1], alphas, launch=c)
                assert torch.equal(sets[0][2], ref), c
    rows = []
    for c, ts in times.items():
        med = statistics.median(ts)
        rows.append({"blocks_per_cu": c[0], "vec_per_lane": c[1], "nontemporal": c[2],
                     "median_us": round(med * 1e3, 2), "min_us": round(min(ts) * 1e3, 2),
                     "GBps_median": round((K + 2) * P * 4 / (med * 1e-3) / 1e9, 1)})
    rows.sort(key=lambda x: x["median_us"])
    for row in rows:
        print(json.dumps(row))


if __name__ == "__main__":
    main()
