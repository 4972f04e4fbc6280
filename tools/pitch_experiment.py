#!/usr/bin/env python3
"""Does the row pitch of the stacked [L, pitch] population layout change the mix rate?
The 10 concurrent streams of a mix (9 reads, 1 write) start at offsets that are multiples of
the pitch; their alignment against the HBM channel / bank interleave decides how evenly the
concurrent requests spread. Runs a full round per pitch, interleaved, in one process."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.population import RingShardPlan  # noqa: E402

P, L, ROUNDS = 25_000_000, 48, 4
eng = get_engine(0)
plan = RingShardPlan(0, 1, L, 4)
alphas = [1.0 / 9] * 8
pads = [0, 64, 256, 1024, 4096, 16384, 65536, 262144, 1 << 20, -(P % (1 << 18)) + (1 << 18)]
res = {}
for pad in pads:
    pitch = P + pad
    models = torch.empty(L, pitch, device="cuda")
    mixed = torch.empty(L, pitch, device="cuda")
    models.normal_()
    srcs = [[models[j, :P] for j in plan.neighbours(i)] for i in range(L)]
    res[pad] = (models, mixed, srcs)
times = {p: [] for p in pads}
for r in range(ROUNDS):
    for pad in pads:
        models, mixed, srcs = res[pad]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(L):
            eng.mix_seq(mixed[i, :P], models[i, :P], srcs[i], alphas)
        e1.record()
        torch.cuda.synchronize()
        times[pad].append(e0.elapsed_time(e1) / L)
for pad in pads:
    med = statistics.median(times[pad])
    print(json.dumps({"pad_floats": pad, "pitch_bytes": (P + pad) * 4, "us_per_mix": round(med * 1e3, 2),
                      "GBps": round(1e9 / (med * 1e-3) / 1e9, 1)}))
