#!/usr/bin/env python3
"""Is the per-allocation placement level (DESIGN §3 "Placement variance") a property of the input
stack, of the output stack, or of the pair? The bench's population layout (a [128, 25M] fp32
`models` stack read, a [128, 25M] `mixed` stack written, K = 8 ring window) allocated as three
candidate input stacks and three output stacks; every (input, output) pairing timed over whole
rounds, interleaved, several passes. Prints one JSON line per pairing and a summary."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

P, L, C = 25_000_000, int(os.environ.get("PROBE_L", "128")), int(os.environ.get("PROBE_C", "3"))
PASSES = int(os.environ.get("PROBE_PASSES", "3"))
eng = get_engine(0)
alphas = [1.0 / 9] * 8
ins = [torch.empty((L, P), device="cuda") for _ in range(C)]
outs = [torch.empty((L, P), device="cuda") for _ in range(C)]
for t in ins:
    t.normal_()
plans = {}
for a in range(C):
    for b in range(C):
        m, o = ins[a], outs[b]
        plans[(a, b)] = [eng.prepare_mix_seq(o[i], m[i], [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)],
                                             alphas) for i in range(L)]
times = {k: [] for k in plans}
for _ in range(PASSES):
    for k, fns in plans.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for fn in fns:
            fn(None)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1e3 / L)
for (a, b), ts in times.items():
    print(json.dumps({"experiment": "tools/probe/placement_pairs.py", "in_stack": a, "out_stack": b,
                      "us_per_mix": [round(t, 2) for t in ts], "median_us": round(statistics.median(ts), 2)}))
med = {k: statistics.median(v) for k, v in times.items()}
print(json.dumps({"experiment": "tools/probe/placement_pairs.py", "summary": True,
                  "by_in": [round(statistics.mean(med[(a, b)] for b in range(C)), 2) for a in range(C)],
                  "by_out": [round(statistics.mean(med[(a, b)] for a in range(C)), 2) for b in range(C)],
                  "best": min(med, key=med.get), "best_us": round(min(med.values()), 2),
                  "worst_us": round(max(med.values()), 2)}))
