#!/usr/bin/env python3
"""Does the size of the allocation a population's stacks live in set their placement level? A
16-device ring (K = 8, 25M) mixed from the first 16 rows of input and output stacks allocated
with 16, 32, 64 and 128 rows; whole rounds, interleaved over passes, in one process (each size
allocated after the previous ones, all held)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

P, L = 25_000_000, 16
eng = get_engine(0)
alphas = [1.0 / 9] * 8
sizes = [int(x) for x in os.environ.get("ALLOC_ROWS", "16,32,64,128,16").split(",")]
plans = []
for k, rows in enumerate(sizes):
    m, o = torch.empty((rows, P), device="cuda"), torch.empty((rows, P), device="cuda")
    m[:L].normal_()
    fns = [eng.prepare_mix_seq(o[d], m[d], [m[(d + j) % L] for j in (-4, -3, -2, -1, 1, 2, 3, 4)], alphas)
           for d in range(L)]
    plans.append((f"{k}:{rows}rows", m, o, fns))
times = {name: [] for name, *_ in plans}
for _ in range(6):
    for name, _m, _o, fns in plans:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for fn in fns:
            fn(None)
        e1.record()
        e1.synchronize()
        times[name].append(e0.elapsed_time(e1) * 1e3 / L)
print(json.dumps({"experiment": "tools/probe/alloc_size.py",
                  **{n: round(statistics.median(t[1:]), 2) for n, t in times.items()}}))
