#!/usr/bin/env python3
"""Resident workgroups per CU for the one-launch CSR population kernel (cfa_mix_population_f32):
the same population buffers (so one placement for every variant) timed with CFA_POP_WG_PER_CU =
1, 2, 4, 8 (8 = the default), interleaved over passes, for the config shapes the kernel serves:
C5 (128 devices x 24 622, ring), C4 (32 x VGG-1 1 071 748, K = 4 window) and the C5 scaling
shape (32 x 25M, ring), the CSR path forced."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import topology as T  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

eng = get_engine(0)
ballast = torch.empty(25 << 30, dtype=torch.float32, device="cuda")  # 100 GiB held: off first-allocation memory
ballast.zero_()
cases = [("C5 128 x 24622 ring", 128, 24_622, T.ring_v4(128, 1)),
         ("C4 32 x 1071748 K=4 window", 32, 1_071_748, [[(d + o) % 32 for o in (-2, -1, 1, 2)] for d in range(32)]),
         ("C5 scaling 32 x 25M ring", 32, 25_000_000, T.ring_v4(32, 1))]
VARIANTS = [int(v) for v in os.environ.get("POP_VARIANTS", "1,2,4,8").split(",")]
for name, D, P, lists in cases:
    models = torch.randn(D, P, device="cuda")
    pr = T.PopulationRound(eng, models)
    pr.set_topology(lists, T.alphas_tf2, use_window=False)
    reps = 50 if P < 2_000_000 else 5
    times = {v: [] for v in VARIANTS}
    for _ in range(5):
        for v in VARIANTS:
            os.environ["CFA_POP_WG_PER_CU"] = str(v)
            pr.run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                pr.run()
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) * 1e3 / reps)
    alg = sum(len(l) + 2 for l in lists) * P * 4
    print(json.dumps({"experiment": "tools/probe/pop_shape.py", "case": name,
                      **{f"wg{v}_us": round(statistics.median(t), 2) for v, t in times.items()},
                      **{f"wg{v}_GBps": round(alg / (statistics.median(t) * 1e-6) / 1e9, 1) for v, t in times.items()}}),
          flush=True)
    del pr, models
os.environ.pop("CFA_POP_WG_PER_CU", None)
