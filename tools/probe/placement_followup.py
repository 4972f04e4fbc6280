#!/usr/bin/env python3
"""Why can a placement-calibrated pair probe at 156 us per mix and then run the bench's rounds
at 161 us? The chosen pair (federated_amd/placement.py) re-timed over whole rounds: as probed
(zero inputs), after the inputs are filled with seeded normal values (what the bench does), with
the two data sets alternating, and over a long back-to-back run (sustained load)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.placement import calibrated_stacks  # noqa: E402

P, L = 25_000_000, 128
eng = get_engine(0)
alphas = [1.0 / 9] * 8
held = []
m, o, rep = calibrated_stacks(L, P, "cuda", eng, 4, 4, candidates=4, hold=held)
fns = [eng.prepare_mix_seq(o[d], m[d], [m[(d + k) % L] for k in (-4, -3, -2, -1, 1, 2, 3, 4)], alphas)
       for d in range(L)]


def rounds(n):
    out = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for fn in fns:
            fn(None)
        e1.record()
        e1.synchronize()
        out.append(round(e0.elapsed_time(e1) * 1e3 / L, 2))
    return out


res = {"placement": rep, "zeros_rejects_held": rounds(4)}
del held
torch.cuda.empty_cache()
res["zeros"] = rounds(4)
m.normal_(generator=torch.Generator(device="cuda").manual_seed(1))
res["normal"] = rounds(4)
m.zero_()
res["zeros_again"] = rounds(4)
m.normal_(generator=torch.Generator(device="cuda").manual_seed(2))
res["normal_again"] = rounds(4)
# sustained: 25 back-to-back rounds without host synchronisation between them
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
evs = [torch.cuda.Event(enable_timing=True) for _ in range(26)]
evs[0].record()
for r in range(25):
    for fn in fns:
        fn(None)
    evs[r + 1].record()
evs[-1].synchronize()
res["sustained_normal"] = [round(evs[r].elapsed_time(evs[r + 1]) * 1e3 / L, 2) for r in range(25)]
# recovery: whole rounds for about 6 s after the frees; medians per 25 rounds
import time  # noqa: E402
traj, t0 = [], time.perf_counter()
while time.perf_counter() - t0 < 6.0:
    traj += rounds(25)
res["after_free_per25"] = [round(statistics.median(traj[i:i + 25]), 2) for i in range(0, len(traj), 25)]
res["after_free_seconds"] = round(time.perf_counter() - t0, 2)
res["medians"] = {k: statistics.median(v) for k, v in res.items() if isinstance(v, list)}
print(json.dumps({"experiment": "tools/probe/placement_followup.py", **res}))
