#!/usr/bin/env python3
"""Per-device mix time across one population round (L devices, stacked layout, given pad):
looks for address-dependent patterns (which devices' bucket windows run slow)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.population import RingShardPlan  # noqa: E402

P = 25_000_000
L = int(sys.argv[1]) if len(sys.argv) > 1 else 128
pad = int(sys.argv[2]) if len(sys.argv) > 2 else 0
eng = get_engine(0)
plan = RingShardPlan(0, 1, L, 4)
alphas = [1.0 / 9] * 8
models = torch.empty(L, P + pad, device="cuda").normal_()
mixed = torch.empty(L, P + pad, device="cuda")
srcs = [[models[j, :P] for j in plan.neighbours(i)] for i in range(L)]
ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(L)] for _ in range(5)]
for r in range(5):
    for i in range(L):
        ev[r][i][0].record()
        eng.mix_seq(mixed[i, :P], models[i, :P], srcs[i], alphas)
        ev[r][i][1].record()
torch.cuda.synchronize()
per = [statistics.median(ev[r][i][0].elapsed_time(ev[r][i][1]) * 1e3 for r in range(1, 5)) for i in range(L)]
base = models.data_ptr()
print(json.dumps({"L": L, "pad": pad, "base_mod_2MB": base % (1 << 21), "median_us": round(statistics.median(per), 1),
                  "min_us": round(min(per), 1), "max_us": round(max(per), 1)}))
print(" ".join(f"{x:.0f}" for x in per))
