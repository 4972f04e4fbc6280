#!/usr/bin/env python3
"""Population layout in HBM, same process/box, sliding-window rounds, interleaved:
stacked rows (pitch = P*4), pitch rounded up to 2 MiB, 2 MiB + 1 MiB, and one allocation per
device. Prints us per mix for each."""
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
MiB2 = (2 << 20) // 4


def stacked(pitch):
    m = torch.empty(L, pitch, device="cuda")
    o = torch.empty(L, pitch, device="cuda")
    m[:, :P].normal_()
    return [m[i, :P] for i in range(L)], [o[i, :P] for i in range(L)]


def separate():
    return [torch.randn(P, device="cuda") for _ in range(L)], [torch.empty(P, device="cuda") for _ in range(L)]


up2 = ((P + MiB2 - 1) // MiB2) * MiB2
layouts = {"stacked_pitch_P": stacked(P), "stacked_pitch_2MiB": stacked(up2),
           "stacked_pitch_2MiB_plus_1MiB": stacked(up2 + MiB2 // 2), "separate_allocs": separate()}


def run(rows, outs):
    for i in range(L):
        eng.mix_seq(outs[i], rows[i], [rows[(i + o) % L] for o in (-4, -3, -2, -1, 1, 2, 3, 4)], a)


times = {k: [] for k in layouts}
for _ in range(R):
    for k, (rows, outs) in layouts.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(rows, outs)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / L)
for k, ts in times.items():
    m = statistics.median(ts)
    print(json.dumps({"layout": k, "us_per_mix": round(m * 1e3, 2), "min_us": round(min(ts) * 1e3, 2),
                      "GBps": round(1e9 / (m * 1e-3) / 1e9, 1)}))
