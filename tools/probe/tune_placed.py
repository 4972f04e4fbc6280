#!/usr/bin/env python3
"""Launch-shape sweep of the K = 8 x 25M mix on placement-calibrated stacks.

The round-1 sweep (tools/tune_mix.py) rotated four separately allocated buffer sets, so every
configuration's samples mixed placement levels (median 163 us against a 150 us minimum). Here the
buckets are one ring population of L devices whose stacks were chosen by the placement probe
(federated_amd/placement.py), and every configuration (workgroups per CU, float4 per lane,
nontemporal policy) runs whole rounds of it, interleaved over passes."""
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.placement import calibrated_stacks  # noqa: E402

P, L, PASSES = 25_000_000, int(os.environ.get("TUNE_L", "32")), int(os.environ.get("TUNE_PASSES", "5"))
H = int(os.environ.get("TUNE_HALF", "4"))  # K = 2 H ring-window neighbours
eng = get_engine(0)
alphas = [1.0 / (2 * H + 1)] * (2 * H)
m, o, rep = calibrated_stacks(L, P, "cuda", eng, H, H, candidates=4)
m.normal_(generator=torch.Generator(device="cuda").manual_seed(3))
srcs = [[m[(d + k) % L] for k in list(range(-H, 0)) + list(range(1, H + 1))] for d in range(L)]
cfgs = list(itertools.product([1, 2, 3, 4], [1, 2, 4], [0, 1]))
times = {c: [] for c in cfgs}
for _ in range(PASSES):
    for c in cfgs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for d in range(L):
            eng.mix_seq(o[d], m[d], srcs[d], alphas, launch=c)
        e1.record()
        e1.synchronize()
        times[c].append(e0.elapsed_time(e1) * 1e3 / L)
print(json.dumps({"experiment": "tools/probe/tune_placed.py", "neighbours": 2 * H, "placement": rep}))
for c in sorted(cfgs, key=lambda c: statistics.median(times[c])):
    med = statistics.median(times[c])
    print(json.dumps({"experiment": "tools/probe/tune_placed.py", "neighbours": 2 * H, "blocks_per_cu": c[0], "vec_per_lane": c[1],
                      "nontemporal": c[2], "median_us": round(med, 2), "min_us": round(min(times[c]), 2),
                      "GBps": round((2 * H + 2) * P * 4 / (med * 1e-6) / 1e9, 1)}))
