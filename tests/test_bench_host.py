"""CPU tests of bench.py's host logic that needs no GPU: the live PMC traffic reader (against a
stand-in `rocprofv3` that writes the counter CSV rocprofv3 writes) and its fallbacks."""
import os
import stat
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FAKE = r'''#!/usr/bin/env python3
import os, sys
args = sys.argv[1:]
d = args[args.index("-d") + 1]
counter = args[args.index("--pmc") + 1]
if os.environ.get("FAKE_ROCPROF_ARGV"):
    with open(os.environ["FAKE_ROCPROF_ARGV"], "a") as fh:
        fh.write(" ".join(args) + "\n")
if os.environ.get("FAKE_ROCPROF_FAIL"):
    sys.exit(3)
os.makedirs(os.path.join(d, "host", "1234"), exist_ok=True)
val = {"FETCH_SIZE": 439498.625, "WRITE_SIZE": 97656.25}[counter]
with open(os.path.join(d, "host", "1234", "pmc_counter_collection.csv"), "w") as fh:
    fh.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n")
    for i in range(6):
        name = '"void (anonymous namespace)::mix_vec_kernel<8, 0, 2, 2>(float*)"'
        fh.write(f"{i},{name},{counter},{val / 2}\n")
        fh.write(f"{i},{name},{counter},{val / 2}\n")  # per-XCD rows of one dispatch
        fh.write(f'{100 + i},"void other_kernel()",{counter},1.0\n')
'''


@pytest.fixture
def fake_rocprof(tmp_path, monkeypatch):
    exe = tmp_path / "rocprofv3"
    exe.write_text(FAKE)
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setenv("PATH", f"{tmp_path}{os.pathsep}{os.environ['PATH']}")
    return exe


def test_live_traffic_reads_and_corrects_the_pmc_passes(fake_rocprof):
    import bench
    val, note = bench.live_traffic(25_000_000, 8, timeout=60)
    # read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB; rows of one dispatch summed
    assert val == pytest.approx(2 * 439498.625 * 1024 + 97656.25 * 1024)
    assert "this run" in note


def test_live_traffic_ring_mode_profiles_the_rank_round(fake_rocprof, monkeypatch, tmp_path):
    """N > 1: the probe child runs the rank's ring round (--ring D) on the rank's slice length."""
    import bench
    argv = tmp_path / "argv.txt"
    monkeypatch.setenv("FAKE_ROCPROF_ARGV", str(argv))
    val, note = bench.live_traffic(3_125_000, 8, timeout=60, ring=128)
    lines = argv.read_text().splitlines()
    assert len(lines) == 2 and all("--params 3125000" in ln and ln.endswith("--ring 128") for ln in lines)
    assert val == pytest.approx(2 * 439498.625 * 1024 + 97656.25 * 1024)
    assert "--ring 128" in note


def test_live_traffic_reports_a_failed_pass(fake_rocprof, monkeypatch):
    import bench
    monkeypatch.setenv("FAKE_ROCPROF_FAIL", "1")
    val, note = bench.live_traffic(25_000_000, 8, timeout=60)
    assert val is None and "failed" in note


def test_live_traffic_without_profiler(monkeypatch, tmp_path):
    import bench
    monkeypatch.setenv("PATH", str(tmp_path))
    val, note = bench.live_traffic(25_000_000, 8, timeout=60)
    assert val is None and "not on PATH" in note


def test_watchdog_ends_a_stuck_run_with_its_phase():
    """A run that never finishes (e.g. one rank stuck in a collective) exits with status 124 and
    names the phase it was in; a run that finishes in time is left alone."""
    import subprocess
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "w = bench.Watchdog(%s, 3); w.enter('timed rounds'); time.sleep(%s); w.done(); print('finished')")
    stuck = subprocess.run([sys.executable, "-c", code % (ROOT, 0.5, 30)], capture_output=True, text=True,
                           timeout=60)
    assert stuck.returncode == 124
    assert "[bench rank 3] FATAL: watchdog" in stuck.stderr and "'timed rounds'" in stuck.stderr
    ok = subprocess.run([sys.executable, "-c", code % (ROOT, 30, 0.1)], capture_output=True, text=True, timeout=60)
    assert ok.returncode == 0 and "finished" in ok.stdout


def test_watchdog_leg_budget_reports_and_exits_with_its_status():
    """An extra N > 1 leg past its own budget runs the leg's on_expire (which prints the line with
    the legs measured so far) and exits with its status, whatever phases were entered inside the
    leg; after end_leg the budget no longer applies."""
    import subprocess
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "w = bench.Watchdog(60, 0)\n"
            "def expire(phase):\n"
            "    print('partial line, stuck in', phase, flush=True); return 0\n"
            "w.leg('devices leg', %s, expire); w.enter('route autotune (devices)'); time.sleep(%s)\n"
            "w.end_leg(); w.enter('after'); time.sleep(%s); w.done(); print('finished')")
    stuck = subprocess.run([sys.executable, "-c", code % (ROOT, 0.5, 30, 0)], capture_output=True, text=True,
                           timeout=60)
    assert stuck.returncode == 0
    assert "partial line, stuck in route autotune (devices)" in stuck.stdout and "finished" not in stuck.stdout
    assert "did not finish within its 0 s budget" in stuck.stderr or "budget" in stuck.stderr
    ok = subprocess.run([sys.executable, "-c", code % (ROOT, 0.5, 0.1, 1.0)], capture_output=True, text=True,
                        timeout=60)
    assert ok.returncode == 0 and "finished" in ok.stdout and "partial" not in ok.stdout
