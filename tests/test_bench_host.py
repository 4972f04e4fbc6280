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


# ---- N > 1 self-launch and the total budget (round 4) ----

def test_child_command_is_the_drivers_torchrun_form():
    import bench
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = bench.child_command(argv, 8, 29555, python="/usr/bin/python3")
    assert cmd[:3] == ["/usr/bin/python3", "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    script = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[script + 1:] == argv  # the caller's arguments, unchanged, after the script


def test_child_env_sets_origin_and_status_and_drops_rank_vars():
    import bench
    base = {"PATH": "/bin", "RANK": "3", "WORLD_SIZE": "8", "LOCAL_RANK": "3", "MASTER_PORT": "1",
            "HSA_ENABLE_IPC_MODE_LEGACY": "0", "OMP_NUM_THREADS": "16"}
    env = bench.child_env(base, 1234.5, "/tmp/status")
    assert "RANK" not in env and "WORLD_SIZE" not in env and "LOCAL_RANK" not in env and "MASTER_PORT" not in env
    assert env[bench.T0_ENV] == "1234.5" and env[bench.STATUS_FILE_ENV] == "/tmp/status"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and env["OMP_NUM_THREADS"] == "16"
    assert env["PYTHONUNBUFFERED"] == "1"
    assert bench.child_env({}, 0.0, "x")["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # the box's hardware-queue setting is never overridden (round 6: no wait parks on a GPU queue)
    assert "GPU_MAX_HW_QUEUES" not in env
    assert bench.child_env({"GPU_MAX_HW_QUEUES": "4"}, 0.0, "x")["GPU_MAX_HW_QUEUES"] == "4"
    assert not hasattr(bench, "set_hw_queues")
    assert bench.hw_queues_report({"GPU_MAX_HW_QUEUES": "4"}) == "4"
    assert bench.hw_queues_report({}) == "unset (HIP default 4)"


def test_lane_reserve_covers_every_plan_share():
    """The lane probe's reservation is the largest per-pair halo demand: N = 2 (both halos between
    one pair) 8 rows, N >= 3 4 rows, params: nothing to exchange."""
    import bench
    P = 25_000_000
    assert bench.lane_reserve_elems(2, 128, 4, 4, P) == 8 * P
    assert bench.lane_reserve_elems(8, 128, 4, 4, P) == 4 * P
    assert bench.lane_reserve_elems(4, 128, 4, 4, P, "params") == 0
    from federated_amd.population import slice_bounds
    assert bench.lane_reserve_elems(4, 128, 4, 4, P, "hybrid", 2) == 8 * slice_bounds(P, 2)[1]


FAKE_TORCHRUN = r'''#!/usr/bin/env python3
import os, sys, time
# stand-in for "python -m torch.distributed.run ... bench.py ARGS": prints what the ranks print
assert sys.argv[1:3] == ["-m", "torch.distributed.run"], sys.argv
mode = os.environ.get("FAKE_MODE", "ok")
print("[rank 1] some stdout chatter", flush=True)
if mode == "hang":
    time.sleep(60)
print('{"metric": "m", "value": 1.0, "n_gpus": 2, "exit_status": %d}' % (5 if mode == "leg" else 0), flush=True)
print('{"second": "line"}', flush=True)
if mode == "leg":
    with open(os.environ["CFA_BENCH_STATUS_FILE"], "w") as fh:
        fh.write("5")
    sys.exit(1)  # torch.distributed.run reports a failed rank as 1
sys.exit(0)
'''


def _self_launch(tmp_path, mode, total=60.0, grace=120.0):
    import subprocess
    fake = tmp_path / "fakepy"
    fake.write_text(FAKE_TORCHRUN)
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    code = ("import sys; sys.path.insert(0, %r); import bench\n"
            "sys.exit(bench.self_launch(['--gpus', '2'], 2, %s, grace=%s, python=%r))" % (ROOT, total, grace, str(fake)))
    env = dict(os.environ, FAKE_MODE=mode)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)


def test_self_launch_relays_exactly_one_line_and_the_status(tmp_path):
    import json
    r = _self_launch(tmp_path, "ok")
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert r.returncode == 0 and len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2
    assert "some stdout chatter" in r.stderr and '"second"' in r.stderr and "launching 2 ranks" in r.stderr
    # rank 0's own status (status file) wins over torch.distributed.run's 1
    r = _self_launch(tmp_path, "leg")
    assert r.returncode == 5 and json.loads(r.stdout.strip())["exit_status"] == 5


def test_self_launch_ends_ranks_that_outlive_the_budget(tmp_path):
    import time as _t
    t = _t.time()
    r = _self_launch(tmp_path, "hang", total=1.0, grace=1.0)
    assert r.returncode == 124 and _t.time() - t < 30
    assert "outlived" in r.stderr and r.stdout.strip() == ""


def test_budget_and_leg_plan_drop_the_last_legs_first():
    import bench
    clock = [100.0]
    b = bench.Budget(420, t0=100.0, clock=lambda: clock[0])
    assert b.left() == 420 and b.allows(420) and not b.allows(421)
    clock[0] = 400.0
    assert b.left() == 120
    assert bench.Budget(0, t0=0.0).left() == float("inf")
    legs = bench.extra_legs(8, 128, "devices")
    assert [n for n, *_ in legs] == ["params", "hybrid2", "weak"]
    assert legs[1] == ("hybrid2", "hybrid", 2) and legs[2] == ("weak", "devices", None)
    assert [n for n, *_ in bench.extra_legs(2, 128, "devices")] == ["params", "weak"]
    assert [n for n, *_ in bench.extra_legs(4, 128, "params", weak_leg=False)] == ["devices", "hybrid2"]
    est = [bench.leg_estimate(n, 8, 20.0, scattered=(n != "weak")) for n, *_ in legs]
    assert est[0] == pytest.approx(45.0) and est[2] == pytest.approx(240.0)
    kept, skipped = bench.plan_within_budget(legs, est, left=170.0, reserve=105.0)
    assert kept == ["params"] and skipped == ["hybrid2", "weak"]
    kept, skipped = bench.plan_within_budget(legs, est, left=400.0, reserve=105.0)
    assert kept == ["params", "hybrid2"] and skipped == ["weak"]
    kept, skipped = bench.plan_within_budget(legs, est, left=1000.0, reserve=105.0)
    assert kept == ["params", "hybrid2", "weak"] and skipped == []


def test_cache_reuse_marking_by_slice_size():
    import bench
    # N = 8 params slice (3.125M fp32 rows): 9 rows = 112.5 MB fit the 256 MiB Infinity Cache
    assert bench.window_fits_cache(bench.leg_slice_P("params", None, 8, 25_000_000), 8)
    # hybrid2 at N = 8 (4 slices of 6.25M): 225 MB, fits; at N = 4 (2 slices of 12.5M): does not
    assert bench.window_fits_cache(bench.leg_slice_P("hybrid", 2, 8, 25_000_000), 8)
    assert not bench.window_fits_cache(bench.leg_slice_P("hybrid", 2, 4, 25_000_000), 8)
    # the devices headline keeps whole 25M buckets: 900 MB windows, no reuse at any N
    assert not bench.window_fits_cache(bench.leg_slice_P("devices", None, 8, 25_000_000), 8)


def test_bench_defaults_put_the_devices_partition_in_the_headline(monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    a = bench.parse()
    assert a.partition == "devices" and a.total_seconds == 420.0 and a.watchdog_seconds is None


def test_record_status_first_writer_wins(tmp_path, monkeypatch):
    import bench
    path = tmp_path / "st"
    monkeypatch.setenv(bench.STATUS_FILE_ENV, str(path))
    bench.record_status(5)
    bench.record_status(0)
    assert path.read_text() == "5"


def test_self_launch_forwards_a_termination_to_the_ranks(tmp_path):
    """An outer time limit that signals the parent ends the launcher (and its ranks) as well; the
    launcher is not detached into a session of its own."""
    import signal
    import subprocess
    import time as _t
    fake = tmp_path / "fakepy"
    fake.write_text(FAKE_TORCHRUN)
    fake.chmod(fake.stat().st_mode | stat.S_IEXEC)
    pidfile = tmp_path / "child.pid"
    code = ("import os, sys; sys.path.insert(0, %r); import bench, subprocess\n"
            "orig = subprocess.Popen\n"
            "def rec(*a, **k):\n"
            "    p = orig(*a, **k); open(%r, 'w').write(str(p.pid)); return p\n"
            "subprocess.Popen = rec\n"
            "sys.exit(bench.self_launch(['--gpus', '2'], 2, 600, python=%r))" % (ROOT, str(pidfile), str(fake)))
    parent = subprocess.Popen([sys.executable, "-c", code], env=dict(os.environ, FAKE_MODE="hang"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    for _ in range(100):
        if pidfile.exists() and pidfile.read_text():
            break
        _t.sleep(0.1)
    child = int(pidfile.read_text())
    assert os.getpgid(child) == os.getpgid(parent.pid)  # same process group as the parent
    _t.sleep(0.5)
    parent.send_signal(signal.SIGTERM)
    out, err = parent.communicate(timeout=60)
    assert parent.returncode == 128 + signal.SIGTERM and "ending the ranks" in err
    _t.sleep(0.2)
    with pytest.raises(ProcessLookupError):
        os.kill(child, 0)


def test_rccl_diagnostics_only_fill_what_is_unset(tmp_path):
    """N > 1 ranks get NCCL_DEBUG=WARN and a per-rank RCCL log file unless the caller set them;
    the tail of that log is what goes into headline_fallback.error / links.error on a failure."""
    import bench
    env = {}
    path = bench.setup_rccl_diagnostics(3, env)
    assert env["NCCL_DEBUG"] == "WARN" and env["NCCL_DEBUG_FILE"] == path and "_r3_" in path
    env = {"NCCL_DEBUG": "INFO", "NCCL_DEBUG_FILE": str(tmp_path / "mine.log")}
    assert bench.setup_rccl_diagnostics(0, env) == str(tmp_path / "mine.log") and env["NCCL_DEBUG"] == "INFO"
    assert bench.setup_rccl_diagnostics(0, {"NCCL_DEBUG_FILE": "/tmp/x.%h.%p"}) is None
    log = tmp_path / "rccl.log"
    log.write_text("x" * 5000 + "\nnode:1:1 [0] NCCL WARN Cuda failure 'invalid device ordinal'\n")
    tail = bench.rccl_log_tail(str(log), limit=200)
    assert tail.endswith("invalid device ordinal'") and len(tail) <= 200
    assert bench.rccl_log_tail(str(tmp_path / "missing")) == "" and bench.rccl_log_tail(None) == ""


def test_decomposition_is_budget_gated_and_never_the_headline():
    """The decomposition sub-legs (exchange only, compute only) run only when the budget left covers
    their estimate; the estimate scales with the headline's own round time."""
    import bench
    est = bench.decomposition_estimate(0.010, 10, 3)
    assert est == pytest.approx(1.5 * 2 * 0.010 * 13 + 5.0)
    assert bench.decomposition_estimate(0.1, 10, 3) > est
    b = bench.Budget(420, t0=0.0, clock=lambda: 410.0)
    assert not b.allows(15.0 + est)  # 10 s left: dropped, reported as skipped: budget
    assert bench.Budget(420, t0=0.0, clock=lambda: 10.0).allows(15.0 + est)


def test_bench_parses_the_route_and_decomposition_flags(monkeypatch):
    import bench
    monkeypatch.setattr("sys.argv", ["bench.py"])
    a = bench.parse()
    assert a.route_tune == "links" and a.link_probe_mb == 64.0 and not a.no_decomposition and a.decomp_steps == 0
    monkeypatch.setattr("sys.argv", ["bench.py", "--route-tune", "wallclock", "--no-decomposition"])
    a = bench.parse()
    assert a.route_tune == "wallclock" and a.no_decomposition
    # the host lane: probed and offered by default, off on request
    monkeypatch.setattr("sys.argv", ["bench.py"])
    a = bench.parse()
    assert a.host_lane == "auto" and a.lane_probe_mb == 256.0
    monkeypatch.setattr("sys.argv", ["bench.py", "--host-lane", "off", "--lane-probe-mb", "64"])
    a = bench.parse()
    assert a.host_lane == "off" and a.lane_probe_mb == 64.0


def _lane_fallback_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from federated_amd import hostlane
        from federated_amd.dist import TorchTransport
        from federated_amd.halo import LANE_IN, LANE_OUT, is_lane_link
        from federated_amd.linkprobe import agree_gloo
        from federated_amd.population import make_ring_shard
        tok = [hostlane.new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        rates = {(a, b): 50.0 for a in range(world) for b in range(world) if a != b}
        rates.update({(a, LANE_OUT): 50.0 for a in range(world)})
        rates.update({(LANE_IN, a): 50.0 for a in range(world)})
        probe = {"plan_rates": rates}
        lane = {"error": None}
        D, P = 16, 4096 + 64
        attempts = []
        real_dir = hostlane.SHM_DIR

        def measure():
            # rank 1's first lane open cannot create its segments (no such directory): HostLane.open
            # raises on every rank, as a full /dev/shm or a refused pin would in the headline
            hostlane.SHM_DIR = "/nonexistent-cfa-lane" if (rank == 1 and not attempts) else real_dir
            attempts.append(1)
            shard, info = make_ring_shard(rank, world, D, 4, 4, P, "cpu", TorchTransport(), None,
                                          link_rates=probe["plan_rates"], lane_token=f"{tok[0]}s{len(attempts)}",
                                          lane_agree=agree_gloo, lane_chunk_elems=256)
            for i in range(shard.plan.L):
                shard.models[i] = torch.full((P,), float(shard.plan.first + i))
            shard.exchange()
            return shard, info
        res, err = bench.headline_with_lane_fallback(measure, agree_gloo, lane, probe)
        shard, info = res
        ok = err is None and info["partition"] == "devices" and not info["route"]["lane"]
        ok &= shard.lane is None and len(attempts) == 2
        ok &= lane["error"] is not None and "host lane" in lane["error"]
        ok &= not any(is_lane_link(k) for k in probe["plan_rates"])
        for i in shard.plan.boundary():  # the lane-free exchange delivered the halo
            g = shard.plan.first + i
            ok &= all(float(s[0]) == float(j) for s, j in zip(shard.sources(i), shard.plan.neighbours(g)))
        q.put((rank, bool(ok), lane["error"]))
    except Exception as exc:
        q.put((rank, False, f"{type(exc).__name__}: {exc}"))
    finally:
        dist.destroy_process_group()


def test_lane_failure_keeps_the_devices_headline():
    """Round-5 review item 2: a host-lane open that fails on ONE rank costs the lane, not the
    devices headline. headline_with_lane_fallback sees the failure on every rank (the open's
    agreement), drops the lane's pseudo-links from the plan's rates, records the error
    (config.host_lane.error) and measures the devices partition again without the lane."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 35300 + (os.getpid() % 997)
    procs = [ctx.Process(target=_lane_fallback_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, msg = q.get(timeout=120)
        res[r] = (ok, msg)
    for p in procs:
        p.join(timeout=30)
    assert all(ok for ok, _ in res.values()), res
    assert "creating the segments failed" in res[0][1]


def test_lane_fallback_without_a_lane_reports_the_error():
    """No lane in the plan: a failed headline is not retried (the caller falls back to params)."""
    import bench
    calls = []

    def measure():
        calls.append(1)
        raise RuntimeError("rccl says no")
    lane, probe = {"error": None}, {"plan_rates": {(0, 1): 50.0, (1, 0): 50.0}}
    res, err = bench.headline_with_lane_fallback(measure, lambda ok: ok, lane, probe)
    assert res is None and "rccl says no" in err and len(calls) == 1 and lane["error"] is None


def test_headline_is_plain_allocation_and_the_calibrated_placement_is_a_leg(monkeypatch):
    """Round-5 review item 4: `value` is measured on plain allocations (what users get); the
    placement-calibrated rounds are the N = 1 leg `legs.placement_calibrated` (asserted on the GPU
    line by tests/test_gpu_bench_contract.py), never the headline."""
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.placement_candidates == 1 and a.placement_leg == 4
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert 'legs_n1["placement_calibrated"]' in src and 'result["legs"] = legs_n1' in src
    # the profiling runs time the headline alone
    assert "--placement-leg 0" in open(os.path.join(ROOT, "tools", "gpu_session.sh")).read()
