"""CPU stress of the host lane's pump thread (federated_amd/csrc/cfa_lane.cpp), built here without
HIP from tests/native/lane_pump_stress.cpp, once plainly and once under ThreadSanitizer: 2 000
rounds of a producer raising chunk words with random pauses against the pump's waits, copies and
group marks, two buffer parities with ack back-pressure, every group's rows checked at its mark;
then the sticky timeout and a destroy that interrupts a pending wait."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "tests", "native", "lane_pump_stress.cpp"),
       os.path.join(ROOT, "federated_amd", "csrc", "cfa_lane.cpp")]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"),
                                reason="needs g++ and the ROCm headers")


def _build(tmp_path, name, flags):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-pthread", "-D__HIP_PLATFORM_AMD__", *flags, f"-I{ROOT}/include",
           "-I/opt/rocm/include", *SRC, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def _run(exe, rounds, seed, timeout):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    p = subprocess.run([exe, str(rounds), str(seed)], capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, f"rc={p.returncode}\n{p.stdout}\n{p.stderr[-4000:]}"
    assert "OK" in p.stdout and "ThreadSanitizer" not in p.stderr, p.stderr[-4000:]
    return p.stdout


def test_lane_pump_stress_plain(tmp_path):
    assert "phase 1: 2000 rounds" in _run(_build(tmp_path, "plain", ["-O2"]), 2000, 5, timeout=240)


@pytest.mark.timeout(600)
def test_lane_pump_stress_tsan(tmp_path):
    assert "phase 1: 1000 rounds" in _run(_build(tmp_path, "tsan", ["-O1", "-g", "-fsanitize=thread"]), 1000, 9,
                                          timeout=540)
