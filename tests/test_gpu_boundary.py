"""Boundary evidence on the GPU: (1) a plain-C program drives libcfa.so through
include/cfa_engine.h with no Python in the loop; (2) the drop-in is re-entrant under the
reference's thread-per-device model (FL_threads_CIFAR100.py:674-681): 8 threads mixing at once
each get the bit-exact result of their own inputs."""
import os
import subprocess
import threading

import numpy as np
import pytest

from conftest import ROOT
from oracle import cfa_oracle as O

pytestmark = pytest.mark.gpu


def test_c_abi_demo_program():
    exe = os.path.join(ROOT, "federated_amd", "lib", "c_abi_demo")
    if not os.path.isfile(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "federated_amd", "csrc"), "demo"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches=0" in r.stdout and "error_rc=-1" in r.stdout and "aliases neighbour" in r.stdout


def test_concurrent_threads_dropin_mixes():
    from federated_amd.consensus._runtime import mixer
    rng = np.random.default_rng(3)
    shapes = [(5, 5, 1, 4), (4,), (5, 5, 4, 8), (8,), (128, 10), (10,)]
    jobs = []
    for t in range(8):
        local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
        nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(1 + t % 4)]
        jobs.append((local, nbrs))
    results = [None] * len(jobs)
    errors = []

    def work(i):
        try:
            local, nbrs = jobs[i]
            a = [1 / (len(nbrs) + 1)] * len(nbrs)
            for _ in range(20):
                out, _ = mixer().mix(local, nbrs, a)
            results[i] = out
        except Exception as exc:  # pragma: no cover - reported below
            errors.append(exc)

    threads = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    for (local, nbrs), out in zip(jobs, results):
        ref = O.tf2_weights(local, nbrs)
        for a, b in zip(out, ref):
            assert np.array_equal(a, b)
