#!/usr/bin/env python3
"""Is the slow placement level tied to a process's first large allocations? The bench layout
([L, 25M] input and output stacks, K = 8 ring-window mixes) allocated as pair A first in the
process, then pair B after 2 x BALLAST_GB of other allocations are held, then pair C after those
are freed; whole rounds of each pair timed, interleaved."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

P, L = 25_000_000, int(os.environ.get("PROBE_L", "128"))
BALLAST = int(os.environ.get("BALLAST_GB", "50"))
eng = get_engine(0)
alphas = [1.0 / 9] * 8


def pair():
    m, o = torch.empty((L, P), device="cuda"), torch.empty((L, P), device="cuda")
    m.normal_()
    return m, o, [eng.prepare_mix_seq(o[d], m[d], [m[(d + k) % L] for k in (-4, -3, -2, -1, 1, 2, 3, 4)], alphas)
                  for d in range(L)]


def rounds(fns, n=3):
    out = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for fn in fns:
            fn(None)
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / len(fns))
    return out


A = pair()
ballast = [torch.empty(BALLAST << 28, dtype=torch.float32, device="cuda") for _ in range(2)]  # 2 x BALLAST GiB
for b in ballast:
    b.zero_()
B = pair()
del ballast
torch.cuda.empty_cache()
C = pair()
t = {"A_first": [], "B_after_ballast": [], "C_after_free": []}
for _ in range(3):
    for k, p in zip(t, (A, B, C)):
        t[k] += rounds(p[2])
print(json.dumps({"experiment": "tools/probe/first_alloc.py", "L": L, "ballast_GiB": 2 * BALLAST,
                  **{k: round(statistics.median(v), 2) for k, v in t.items()},
                  "raw": {k: [round(x, 1) for x in v] for k, v in t.items()}}))
