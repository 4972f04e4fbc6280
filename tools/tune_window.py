#!/usr/bin/env python3
"""Launch-shape sweep of the sliding-window pass (cfa_mix_window_f32, hl = hr = 4, P = 25M):
pass size B, vectors per lane, store policy (sc1 buffer store vs nt store), workgroups per CU.
Reports per-pass time, the algorithmic rate (B devices x 1 GB) and the HBM rate of the bytes a
pass must move ((B + 8) reads + B writes of 100 MB). Interleaved rounds, one process (the
kernel reads its CFA_WINDOW_* overrides at every launch)."""
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

P, L, R, H = 25_000_000, 32, 3, 4
eng = get_engine(0)
m = torch.empty(L, P, device="cuda").normal_()
o = torch.empty(L, P, device="cuda")
al = [1.0 / 9] * 8


def passes(B):
    for s in range(0, L - B + 1, B):
        rows = [m[(s + k - H) % L] for k in range(B + 2 * H)]
        eng.mix_window([o[s + b] for b in range(B)], rows, [al] * B, H, H)


cfgs = list(itertools.product(*(tuple(int(x) for x in os.environ.get(k, d).split(",")) for k, d in (("TW_B", "4,8"), ("TW_VEC", "1,2"), ("TW_SC1", "0,1"), ("TW_BPC", "1,2,4")))))
times = {c: [] for c in cfgs}
for _ in range(R):
    for c in cfgs:
        B, vec, sc1, bpc = c
        os.environ["CFA_WINDOW_VEC"], os.environ["CFA_WINDOW_SC1"] = str(vec), str(sc1)
        os.environ["CFA_WINDOW_BLOCKS_PER_CU"] = str(bpc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        passes(B)
        e1.record()
        torch.cuda.synchronize()
        times[c].append(e0.elapsed_time(e1) / (L // B))
res = []
for c, ts in times.items():
    B = c[0]
    us = statistics.median(ts) * 1e3
    res.append({"B": B, "vec": c[1], "sc1": c[2], "blocks_per_cu": c[3], "us_per_pass": round(us, 1),
                "algorithmic_GBps": round(B * 10 * P * 4 / (us * 1e-6) / 1e9, 1),
                "hbm_GBps": round((2 * B + 2 * H) * P * 4 / (us * 1e-6) / 1e9, 1)})
for r in sorted(res, key=lambda r: -r["algorithmic_GBps"]):
    print(json.dumps(r), flush=True)
