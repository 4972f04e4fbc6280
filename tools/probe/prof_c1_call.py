#!/usr/bin/env python3
"""cProfile of the C1 drop-in call (TF1 cfa.py getFederatedWeight, 2NN, 4 devices, N = 2) with
the protocol sleeps off: where the host time of one call goes, by function."""
import cProfile
import os
import pstats
import sys
import tempfile

os.environ["FEDERATED_AMD_PAUSE_SCALE"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from federated_amd.consensus import cfa  # noqa: E402

os.chdir(tempfile.mkdtemp())
rng = np.random.default_rng(0)
shapes = [(512, 32), (32,), (32, 8), (8,)]
K, N = 4, 2
models = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
procs = [cfa.CFA_process(True, K, j, N) for j in range(K)]
for j in range(K):
    W1, b1, W2, b2 = models[j]
    procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), 1.0)
p = procs[1]
W1, b1, W2, b2 = models[1]


def call():
    p.getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), 1.0)


for _ in range(50):
    call()
pr = cProfile.Profile()
pr.enable()
for _ in range(500):
    call()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
