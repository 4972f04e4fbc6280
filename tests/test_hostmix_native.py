"""CPU test of the drop-in host pipeline ``cfa_host_mix_f32`` (federated_amd/csrc/cfa_hostmix.cpp,
SURVEY §8 f2) itself, not only its copy pool.

The product source is compiled with g++ against tests/native/hostmix_stub: HIP streams emulated
by worker threads (kernels and events run asynchronously, in order), and the two sequential-mix
kernels it launches evaluated on the host. tests/native/hostmix_stress.cpp then calls it from
several threads at once (the reference's one thread per device,
TF2 CIFAR100_dataset/...FL_threads_CIFAR100.py:674-681) with random layer layouts, fan-ins,
chunk sizes, copy-thread counts and divisors, on per-caller and shared streams, and checks every
output bit for bit against the sequential rule (consensus_v3.py:153-155,
parameter_server_v2.py:159-161). Plain and under ThreadSanitizer. Round 2's pipeline crashes
under the same stress (its copy pool's double-counted helper).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def _build(tmp_path, name, flags):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-pthread", "-ffp-contract=off", *flags,
           f"-I{os.path.join(NATIVE, 'hostmix_stub')}", f"-I{os.path.join(ROOT, 'include')}",
           f"-I{os.path.join(ROOT, 'federated_amd', 'csrc')}",
           os.path.join(ROOT, "federated_amd", "csrc", "cfa_hostmix.cpp"),
           os.path.join(NATIVE, "hostmix_stub", "hostmix_stub.cpp"), os.path.join(NATIVE, "hostmix_stress.cpp"),
           "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def _run(exe, callers, iters, seed, timeout):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([exe, str(callers), str(iters), str(seed)], capture_output=True, text=True, timeout=timeout,
                       env=env)
    assert p.returncode == 0, f"rc={p.returncode}\n{p.stdout}\n{p.stderr[-4000:]}"
    assert p.stdout.startswith(f"OK {callers} callers x {iters} calls")
    assert "ThreadSanitizer" not in p.stderr


def test_host_pipeline_concurrent_callers_plain(tmp_path):
    exe = _build(tmp_path, "plain", ["-O2"])
    for seed in (1, 2, 3):
        _run(exe, 4, 300, seed, timeout=120)


@pytest.mark.timeout(600)  # about 30 s on 8 CPUs; headroom over pytest.ini's 300 s on a slower host
def test_host_pipeline_concurrent_callers_tsan(tmp_path):
    _run(_build(tmp_path, "tsan", ["-O1", "-g", "-fsanitize=thread"]), 4, 150, 5, timeout=540)
