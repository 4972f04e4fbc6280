"""CPU stress test of the host copy pool behind cfa_host_mix_f32.

The pool (federated_amd/csrc/cfa_copypool.h) is built here without HIP from
tests/native/copypool_stress.cpp, once plainly and once under ThreadSanitizer, and run for
100 k pool runs whose helper counts alternate 1/3/7/15 with random job counts, then with four
concurrent callers (the reference's one-thread-per-device callers,
TF2 CIFAR100_dataset/federated_learning_keras_consensus_FL_threads_CIFAR100.py:674-681), then
through the bounded-wait (broken pool) path. Round 2's pool deadlocked under exactly this
alternation: its workers read the generation and the helper count as two loads.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "copypool_stress.cpp")
INC = os.path.join(ROOT, "federated_amd", "csrc")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _build(tmp_path, name, flags):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-pthread", *flags, f"-I{INC}", SRC, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def _run(exe, runs, seed, timeout):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    p = subprocess.run([exe, str(runs), str(seed)], capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, f"rc={p.returncode}\n{p.stdout}\n{p.stderr[-4000:]}"
    assert "OK" in p.stdout
    assert "ThreadSanitizer" not in p.stderr, p.stderr[-4000:]
    return p.stdout


def test_copypool_stress_plain(tmp_path):
    out = _run(_build(tmp_path, "plain", ["-O2"]), 100000, 7, timeout=240)
    assert "phase 1: 100000 runs, 15 workers" in out


@pytest.mark.timeout(900)  # 1-2 minutes on 8 CPUs; headroom over pytest.ini's 300 s on a slower host
def test_copypool_stress_tsan(tmp_path):
    out = _run(_build(tmp_path, "tsan", ["-O2", "-g", "-fsanitize=thread"]), 100000, 11, timeout=840)
    assert "phase 1: 100000 runs, 15 workers" in out
