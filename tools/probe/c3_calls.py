#!/usr/bin/env python3
"""Per-call latency of the GPU pieces of one CFA-GE drop-in call at config 3's shapes (CNN,
P = 1 488, 2 neighbours, 24 samples of 512 inputs): the stage-1 TF1 mix, the gradients at the
neighbours' models (one batched launch), and the MEWMA update of model and saved states, with
the numpy restatement of each beside it (oracle, same run). Medians over 300 calls.
--signal-off: end each call with hipStreamSynchronize instead of the completion word."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from federated_amd.consensus import _runtime as R  # noqa: E402
from federated_amd.consensus import _tf1_models  # noqa: E402
from oracle import cfa_oracle as O  # noqa: E402

if "--signal-off" in sys.argv:
    R.SIGNAL_COMPLETION = False


def med(fn, n=300):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


rng = np.random.default_rng(3)
shapes = [(16, 1, 8), (8,), (168, 8), (8,)]
mk = lambda dt=np.float32: [(rng.standard_normal(s) * 0.1).astype(dt) for s in shapes]
local, nbrs = mk(), [mk(), mk()]
x = rng.standard_normal((24, 512)).astype(np.float32)
y = np.eye(8, dtype=np.float32)[rng.integers(0, 8, 24)]
N = 2
states = [np.zeros(s + (N,), np.float64) for s in shapes]
grads = [mk(np.float64), mk(np.float64)]
mx = R.mixer()
res = {"experiment": "tools/probe/c3_calls.py", "P": 1488, "n": 2, "signal_completion": R.SIGNAL_COMPLETION}
res["stage1_mix_tf1_us"] = med(lambda: mx.mix_tf1(local, nbrs, [0.5, 0.5]))
res["numpy_stage1_us"] = med(lambda: O.tf1_mix(local, nbrs, 1.0, [np.float64(0.5)] * 2))
res["gradients_batched_us"] = med(lambda: _tf1_models.gradients_batched(1, x, y, nbrs, stride=5))
res["numpy_gradients_us"] = med(lambda: [O.tf1_cnn_grads(x, y, *m, 5) for m in nbrs], 30)
res["mewma_tf1_us"] = med(lambda: mx.mewma_tf1(local, states, grads, 0.99, (0.1, 0.1, 0.2, 0.2), False, True))
print(json.dumps(res))
