#!/usr/bin/env python3
"""Launch-shape sweep of the one-launch ring round (cfa_mix_ring_round_f32) at the population
sizes it serves: C4 (32 devices x 1 071 748, K = 4, FL_threads_CIFAR100.py:160-170) and larger
buckets. The window kernels read their shape from the environment at every launch
(CFA_WINDOW_BLOCKS_PER_CU, CFA_WINDOW_VEC; results identical), so one process times every shape on
the same stacks, interleaved over passes. Prints one JSON line per (case, shape): median us per
round and the algorithmic rate (every device's (K + 2) P 4 bytes)."""
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

CASES = [(32, 1_071_748, 2, 2), (32, 4_000_000, 2, 2), (128, 3_125_056, 4, 4), (32, 25_000_000, 4, 4)]
BPC = [int(x) for x in os.environ.get("RR_BPC", "2,4,6,8,12,16").split(",")]
VEC = [int(x) for x in os.environ.get("RR_VEC", "1,2").split(",")]
PASSES = int(os.environ.get("RR_PASSES", "7"))
eng = get_engine(0)
for D, P, hl, hr in CASES:
    models = torch.empty((D, P), dtype=torch.float32, device="cuda").normal_(generator=torch.Generator(device="cuda").manual_seed(5))
    out = torch.empty_like(models)
    K = hl + hr
    alphas = torch.full((D,), 1.0 / (K + 1), dtype=torch.float32, device="cuda")
    shapes = list(itertools.product(BPC, VEC))
    times = {s: [] for s in shapes}

    def run(s):
        os.environ["CFA_WINDOW_BLOCKS_PER_CU"], os.environ["CFA_WINDOW_VEC"] = str(s[0]), str(s[1])
        eng.ring_round(out, models, alphas, hl, hr)

    for s in shapes:
        run(s)
    for _ in range(PASSES):
        for s in shapes:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            run(s)  # warm the shape
            e0.record()
            for _ in range(3):
                run(s)
            e1.record()
            e1.synchronize()
            times[s].append(e0.elapsed_time(e1) * 1e3 / 3)
    alg = D * (K + 2) * P * 4
    for s in sorted(shapes, key=lambda s: statistics.median(times[s])):
        us = statistics.median(times[s])
        print(json.dumps({"experiment": "tools/probe/ring_round_shape.py", "devices": D, "P": P, "hl": hl, "hr": hr,
                          "blocks_per_cu": s[0], "vec": s[1], "us_per_round": round(us, 2),
                          "algorithmic_GBps": round(alg / (us * 1e-6) / 1e9, 1),
                          "default": s == (6, 1)}), flush=True)
    del models, out
    torch.cuda.empty_cache()
