#!/usr/bin/env python3
"""Benchmark: device-resident CFA reduction of K neighbour fp32 buckets on MI355X.

Metric (BASELINE.json): "device-resident GB/s, CFA reduce of K neighbour fp32 param buckets;
1/2/4/8 GPU". Workload (BASELINE.json north_star target): 8 neighbour buckets x 25M fp32 params
mixed into each device's local model (the TF2 sequential CFA rule, eps = 1/(K+1),
consensus_v3.py:145,153-155), for every device of a simulated population of D = 128 devices on
a wrap-around ring window of K = 8 neighbours. One step = one consensus round of the whole
population.

Scaling (SURVEY §8 e: "Strong scaling, fixed population"): the population stays D = 128 for
every N. The headline at every N is the ``devices`` partition, north_star's "when devices are
sharded": contiguous device blocks, one per rank; a round is the routed halo exchange of the 2x4
boundary buckets of each rank (federated_amd/halo.py: direct plus relayed xGMI paths over RCCL,
sent row by row) overlapped with the interior mixes, each boundary device mixing as soon as the
rows it reads have landed. Beside it, in ``partitions``, the same population, steps and clock on
the other partitions: ``params`` (every rank a 1/N element slice of every bucket, no exchange),
``hybrid2`` (from N = 4: 2 device blocks x N/2 slices) and ``weak`` (128 devices per GPU,
D = 128 N). A leg whose ring window ((K + 1) rows of the rank's slice) fits the 256 MiB Infinity
Cache is marked ``cache_reuse: true`` and also timed with its mixes in a scattered order
(``value_scattered``: consecutive mixes share no rows), since its algorithmic-byte rate is then
partly served by the cache and is not an HBM fraction. ``--devices-per-gpu L`` makes the weak
form the headline (D = L*N).

The headline runs on plain allocations, what every user of the library gets (round 6). At N = 1
the same rounds are also timed on placement-calibrated stacks (``legs.placement_calibrated``,
``--placement-leg``, federated_amd/placement.py: the fastest of 4 allocations per stack, probed
with the same mix), reported beside the headline and never as ``value``.

value = algorithmic bytes of all mixes on all ranks / max-over-ranks wall time, with
algorithmic bytes = (K + 2) * P * 4 per device mix (K neighbour reads + local read + output
write). Inputs are resident in HBM when the timed region starts.

Launch: ``python bench.py [--gpus N --steps K --warmup W]``. With N > 1 and no RANK/WORLD_SIZE in
the environment the bench launches its own ranks: ``python -m torch.distributed.run --nnodes=1
--nproc-per-node N --master-addr 127.0.0.1`` as a child process, before anything touches the GPU;
the parent relays rank 0's JSON line and exits with the run's status. Under an external
torch.distributed.run it runs as the rank it is given.

Time: ``--total-seconds`` (default 420) bounds the whole run from the first launch: the headline
is always measured; the extra legs, the CPU baselines, the PMC passes and the e2e leg each run
only if the budget left covers their estimate, otherwise they are listed as ``skipped: budget``.

Exit status: 0 = the line is complete; 3 = the transport the headline needs (RCCL) could not be
opened on every rank, or the exchanging headline raised on every rank (the line is printed with
the ``params`` partition, which exchanges nothing, as ``value`` and ``config.headline_fallback``
saying why); 5 = the line is printed but an extra
leg failed, ran out of its budget or lost a peer (named in ``partitions``); 124 = the watchdog
ended a run stuck in its headline (no line). Self-launched, the parent returns the same status.
"""
from __future__ import annotations

import argparse
import json
import statistics
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
KERNEL = "mix_vec_kernel"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--params", type=int, default=25_000_000, help="P, fp32 params per bucket")
    p.add_argument("--neighbours", type=int, default=8, help="K (even: ring window K/2 per side)")
    p.add_argument("--devices", type=int, default=128,
                   help="simulated devices in the whole population (fixed for every N: strong scaling)")
    p.add_argument("--devices-per-gpu", type=int, default=None,
                   help="weak scaling instead: this many devices per GPU (population = N x this)")
    p.add_argument("--partition", default="devices", choices=["devices", "params", "hybrid"],
                   help="the headline's partition: devices (default; contiguous device blocks + routed halo "
                        "exchange), params (every rank a 1/N element slice of every bucket, no exchange), "
                        "hybrid (--device-groups blocks, each split over N/groups slices)")
    p.add_argument("--device-groups", type=int, default=None)
    p.add_argument("--no-relay", action="store_true", help="halo on the direct links only")
    p.add_argument("--no-stages", action="store_true",
                   help="whole halo in one exchange step (boundary devices wait for all of it)")
    p.add_argument("--no-extra-legs", "--no-params-leg", dest="no_extra_legs", action="store_true",
                   help="N > 1: skip the other partitions' measurements (devices, hybrid2) beside the headline")
    p.add_argument("--route-tune", default="links", choices=["links", "wallclock", "none"],
                   help="N > 1: how the halo route is chosen. links (default): plan with per-link costs from "
                        "the link probe's measured rates (the relayed plan is kept only where it shortens the "
                        "predicted critical path); wallclock: round 4's autotune, the relayed plan against "
                        "the direct-only plan over a few timed rounds each; none: uniform link costs")
    p.add_argument("--no-autotune", action="store_true",
                   help="N > 1: same as --route-tune none")
    p.add_argument("--link-probe-mb", type=float, default=64.0,
                   help="N > 1: message size (MB) of the per-link probe run before the route is planned "
                        "(federated_amd/linkprobe.py; 0 = no probe)")
    p.add_argument("--host-lane", default="auto", choices=["auto", "off"],
                   help="auto: probe the host lane (halo pieces over PCIe through pinned shared host memory, "
                        "federated_amd/hostlane.py) after the link probe and offer it to the route plan; off: xGMI only")
    p.add_argument("--lane-probe-mb", type=float, default=256.0,
                   help="MB each rank sends over the host lane per probe round")
    p.add_argument("--no-decomposition", action="store_true",
                   help="N > 1: skip the exchange-only / compute-only sub-legs of the headline round")
    p.add_argument("--decomp-steps", type=int, default=0,
                   help="timed rounds of each decomposition sub-leg (0 = min(--steps, 10))")
    p.add_argument("--no-weak-leg", action="store_true",
                   help="N > 1: skip the weak-scaling reference leg (--devices devices per GPU)")
    p.add_argument("--transport", default="rccl", choices=["rccl", "torch"])
    p.add_argument("--allow-fallback", action="store_true",
                   help="if the requested transport cannot open, fall back to torch.distributed "
                        "(nccl, then gloo) and mark the line non-comparable instead of exiting")
    p.add_argument("--p2p-channels", type=int, default=None,
                   help="NCCL_NCHANNELS_PER_PEER for the RCCL communicator (default: RCCL's own)")
    p.add_argument("--cpu-pool-seconds", type=float, default=8.0,
                   help="bounded sample of the process-pool CPU baseline (0 = skip)")
    p.add_argument("--window-batch", type=int, default=0,
                   help="B > 0: mix B consecutive devices per cfa_mix_window_f32 pass (each window row "
                        "loaded once); 0 (default) = one streaming mix per device, the judged kernel")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=None,
                   help="PMC traffic summary (default profiles/r01_pmc_traffic.json, or "
                        "profiles/r01_window_pmc_traffic.json with --window-batch)")
    p.add_argument("--no-live-traffic", action="store_true",
                   help="do not measure roofline.traffic with rocprofv3 PMC passes in this run (N = 1: "
                        "the dominant mix's bucket shape; N > 1: rank 0's ring round); the committed "
                        "profiles/ value is reported instead")
    p.add_argument("--e2e", dest="e2e", action="store_true", default=True,
                   help="(default at N = 1) also measure the host-resident path on rank 0: the same mix with "
                        "the buckets in pinned host memory, serial H2D + mix + D2H, chunk-pipelined, and "
                        "zero-copy over PCIe (reported under \"e2e\", never as value)")
    p.add_argument("--no-e2e", dest="e2e", action="store_false")
    p.add_argument("--placement-candidates", type=int, default=1,
                   help="the headline's stacks: allocate each population stack this many times and keep the "
                        "fastest, timed with the population's own mix before the timed region "
                        "(federated_amd/placement.py; 1 = plain allocation, the default: what users get)")
    p.add_argument("--placement-leg", type=int, default=4,
                   help="N = 1: also time the headline's rounds on stacks calibrated over this many candidates "
                        "(legs.placement_calibrated; 0 or 1 = skip)")
    p.add_argument("--placement-release", action="store_true",
                   help="return the rejected placement candidates to the driver (then wait out its "
                        "background scrub) instead of leaving them in torch's caching allocator")
    p.add_argument("--total-seconds", type=float, default=420.0,
                   help="budget of the whole run from its first launch (0 = none): the headline always runs; "
                        "extra legs, CPU baselines, PMC passes and the e2e leg only while the budget left covers "
                        "their estimate (else listed as skipped: budget)")
    p.add_argument("--watchdog-seconds", type=float, default=None,
                   help="end the run with status 124 and the phase it was in if it has not finished "
                        "after this long (a collective that never completes; default --total-seconds + 90; "
                        "0 = off)")
    p.add_argument("--leg-seconds", type=float, default=240.0,
                   help="N > 1: cap on each extra leg's budget (the total budget left caps it too); a leg that "
                        "has not finished by then is reported as an error in the line, which is then "
                        "printed with the legs measured so far (exit status 5; 0 = no per-leg cap)")
    return p.parse_args()


STATUS_FILE_ENV = "CFA_BENCH_STATUS_FILE"  # self-launch: where rank 0 leaves the run's exit status
T0_ENV = "CFA_BENCH_T0"  # self-launch: the parent's start (epoch seconds), the budget's origin
EXIT_TRANSPORT, EXIT_LEG, EXIT_WATCHDOG = 3, 5, 124


def record_status(code: int) -> None:
    """Leave the run's exit status where a self-launching parent reads it (torch.distributed.run
    itself only reports 0 or 1). The first status written wins."""
    path = os.environ.get(STATUS_FILE_ENV)
    if not path:
        return
    try:
        fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644)
    except OSError:
        return
    with os.fdopen(fd, "w") as fh:
        fh.write(str(int(code)))


def wait_for_status(seconds: float) -> None:
    """A rank other than 0 about to leave early: wait until rank 0 has recorded the run's status
    (self-launched runs), else ``seconds``, so rank 0 is not ended before its line is printed."""
    path = os.environ.get(STATUS_FILE_ENV)
    end = time.monotonic() + seconds
    while time.monotonic() < end:
        if path and os.path.exists(path):
            time.sleep(0.5)  # the line is printed before the status is recorded
            return
        time.sleep(0.1)


def run_origin() -> float:
    """Epoch seconds the run started: the self-launching parent's start when there is one. Only
    handed between the parent and the ranks; every deadline is measured on the monotonic clock
    from ``monotonic_origin`` (a stepped system clock moves neither)."""
    try:
        return float(os.environ[T0_ENV])
    except (KeyError, ValueError):
        return time.time()


def monotonic_origin(t0_epoch: float) -> float:
    """The run's origin on ``time.monotonic``'s scale: the epoch origin converted once, at start-up."""
    return time.monotonic() - max(0.0, time.time() - float(t0_epoch))


class Budget:
    """The whole run's time budget (``--total-seconds``) from ``t0`` (on ``clock``'s scale: monotonic
    seconds, see ``monotonic_origin``)."""

    def __init__(self, total: float, t0: float = None, clock=time.monotonic):
        self.total, self.clock = float(total), clock
        self.t0 = clock() if t0 is None else float(t0)

    def left(self) -> float:
        if self.total <= 0:
            return float("inf")
        return self.total - (self.clock() - self.t0)

    def allows(self, seconds: float) -> bool:
        return self.left() >= seconds


def extra_legs(world: int, devices: int, headline: str, weak_leg: bool = True):
    """The N > 1 legs measured beside the headline, in the order they run (and are dropped when the
    budget runs short: the last ones first): [(name, partition, device groups or None)]."""
    legs = [(part, part, None) for part in ("devices", "params") if part != headline]
    if world >= 4 and devices % 2 == 0 and headline != "hybrid":
        legs.append(("hybrid2", "hybrid", 2))
    if weak_leg:
        legs.append(("weak", "devices", None))
    return legs


def leg_estimate(name: str, world: int, headline_seconds: float, scattered: bool = False) -> float:
    """Seconds a leg is expected to take, from the headline's own build + autotune + timed rounds
    (same population; the weak leg holds N times the devices per rank), with a 1.5x margin and a
    second timed pass for a cache-reuse leg's scattered order."""
    work = float(world) if name == "weak" else 1.0
    return 1.5 * headline_seconds * work * (1.5 if scattered else 1.0)


def plan_within_budget(legs, estimates, left: float, reserve: float):
    """Which legs fit: walks ``legs`` in order, keeping each whose estimate fits in what is left
    after ``reserve`` (the report's own share) and the legs kept before it. Returns (kept,
    skipped) name lists. Host logic of the budget; at run time each leg is re-checked against the
    clock (and agreed across ranks) just before it starts."""
    kept, skipped = [], []
    for (name, *_), est in zip(legs, estimates):
        if left - reserve >= est:
            kept.append(name)
            left -= est
        else:
            skipped.append(name)
    return kept, skipped


class Watchdog:
    """Ends the process (status 124) with the phase it was stuck in if the run has not finished in
    time. A collective that never completes on one rank (a peer that died inside RCCL, a
    mismatched exchange) otherwise hangs every rank until an outer limit kills the job without
    saying where; torch.distributed.run tears the other ranks down once this one exits."""

    def __init__(self, seconds: float, rank: int, t0: float = None):
        import threading
        self.phase, self.rank, self._done = "start-up", rank, threading.Event()
        self.t0 = time.monotonic() if t0 is None else t0  # monotonic scale (monotonic_origin)
        self._leg = None  # (deadline, budget, on_expire) of a phase entered with its own budget
        self.seconds = seconds
        threading.Thread(target=self._watch, daemon=True).start()

    def _watch(self):
        while not self._done.wait(0.25):
            now = time.monotonic()
            leg = self._leg
            if leg is not None and now > leg[0]:
                print(f"[bench rank {self.rank}] watchdog: phase '{self.phase}' did not finish within its "
                      f"{leg[1]:.0f} s budget", file=sys.stderr, flush=True)
                code = leg[2](self.phase)
                record_status(code)
                os._exit(code)
            if self.seconds > 0 and now - self.t0 > self.seconds:
                print(f"[bench rank {self.rank}] FATAL: watchdog: not finished after {self.seconds:.0f} s, "
                      f"stuck in phase '{self.phase}'", file=sys.stderr, flush=True)
                record_status(EXIT_WATCHDOG)
                os._exit(EXIT_WATCHDOG)

    def enter(self, phase: str) -> None:
        self.phase = phase

    def leg(self, phase: str, budget: float, on_expire) -> None:
        """Enter ``phase`` with a budget of its own (seconds, 0 = none) that holds until ``end_leg``
        whatever phases are entered meanwhile: if it runs out, ``on_expire(phase)`` runs on the
        watchdog thread and its return value is the exit status (the N > 1 bench's extra legs: the
        headline is already measured, so a leg stuck in a collective is reported in the line instead
        of losing the whole run)."""
        self.phase = phase
        self._leg = (time.monotonic() + budget, budget, on_expire) if budget > 0 else None

    def end_leg(self) -> None:
        self._leg = None

    def done(self) -> None:
        self._done.set()


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def child_command(argv, n: int, port: int, python: str = None) -> list:
    """argv of the self-launched ranks: the driver's own N > 1 form (torch.distributed.run, one
    node, N ranks, rendezvous on 127.0.0.1) around this script with the caller's arguments."""
    return [python or sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def child_env(base: dict, t0: float, status_file: str) -> dict:
    """The self-launched ranks' environment: the caller's, minus its rank variables, plus the run's
    origin and status file. ``GPU_MAX_HW_QUEUES`` is left as the box exports it (round 6: nothing
    in a round waits on a GPU queue any more, so the pool's 4 queues carry it)."""
    env = dict(base)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env[T0_ENV] = repr(float(t0))
    env[STATUS_FILE_ENV] = status_file
    env["PYTHONUNBUFFERED"] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL on this pool: dmabuf IPC only
    return env


def hw_queues_report(environ=None) -> str:
    """``GPU_MAX_HW_QUEUES`` as the run sees it (never set by the bench)."""
    env = os.environ if environ is None else environ
    v = env.get("GPU_MAX_HW_QUEUES")
    return v if v else "unset (HIP default 4)"


def setup_rccl_diagnostics(rank: int, environ=None):
    """N > 1, before anything initialises RCCL: NCCL_DEBUG=WARN when unset, and RCCL's log in a
    per-rank file when NCCL_DEBUG_FILE is unset, so that the text of RCCL's own warning can go into
    the line when opening the communicator or a collective fails (``rccl_log_tail``). Returns the
    log's path (None when the caller's NCCL_DEBUG_FILE has a %-pattern)."""
    import tempfile
    env = os.environ if environ is None else environ
    env.setdefault("NCCL_DEBUG", "WARN")
    if env.get("NCCL_DEBUG_FILE"):
        path = env["NCCL_DEBUG_FILE"]
        return None if "%" in path else path
    path = os.path.join(tempfile.gettempdir(), f"cfa_rccl_r{rank}_{os.getpid()}.log")
    env["NCCL_DEBUG_FILE"] = path
    return path


def rccl_log_tail(path, limit: int = 1500) -> str:
    """The last ``limit`` bytes of RCCL's log (its warnings), or ''."""
    if not path:
        return ""
    try:
        with open(path, "rb") as fh:
            fh.seek(0, 2)
            n = fh.tell()
            fh.seek(max(0, n - limit))
            data = fh.read()
    except OSError:
        return ""
    return data.decode("utf-8", "replace").strip()


def self_launch(argv, n: int, total_seconds: float, grace: float = 120.0, python: str = None) -> int:
    """Run the N ranks as a child ``torch.distributed.run`` (never an exec: the parent has not
    touched the GPU, and exits with the child's status), relay rank 0's JSON line to stdout and
    every other line of the child's stdout to stderr, and end the launcher (and with it the ranks)
    if it outlives the total budget by ``grace`` seconds or this process is signalled. Returns the run's exit status: rank 0's own
    (status file) when it left one, else the launcher's."""
    import signal
    import subprocess
    import tempfile
    import threading
    t0 = time.time()
    fd, status_file = tempfile.mkstemp(prefix="cfa_bench_status_")
    os.close(fd)
    os.unlink(status_file)  # created by the first rank that records a status
    cmd = child_command(argv, n, free_port(), python)
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    # the launcher stays in this process's group, so an outer time limit that signals the group
    # (coreutils timeout does) reaches every rank too
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=child_env(os.environ, t0, status_file),
                            text=True, bufsize=1)
    killed = threading.Event()

    def end_child():
        """SIGTERM to the launcher (torch.distributed.run ends its ranks on it), SIGKILL after 15 s."""
        for sig in (signal.SIGTERM, signal.SIGKILL):
            try:
                proc.send_signal(sig)
            except ProcessLookupError:
                return
            try:
                proc.wait(timeout=15)
                return
            except subprocess.TimeoutExpired:
                continue

    def kill_group():
        killed.set()
        print(f"[bench] FATAL: the ranks outlived the {total_seconds:.0f} s budget by {grace:.0f} s; "
              "ending them", file=sys.stderr, flush=True)
        end_child()

    def on_signal(signum, frame):
        print(f"[bench] signal {signum}: ending the ranks", file=sys.stderr, flush=True)
        end_child()
        os._exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, on_signal)

    timer = None
    if total_seconds > 0:
        timer = threading.Timer(total_seconds + grace, kill_group)
        timer.daemon = True
        timer.start()
    relayed = 0
    for line in proc.stdout:
        if line.startswith("{") and relayed == 0:
            sys.stdout.write(line)
            sys.stdout.flush()
            relayed += 1
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = proc.wait()
    if timer is not None:
        timer.cancel()
    status = None
    try:
        with open(status_file) as fh:
            status = int(fh.read().strip())
        os.unlink(status_file)
    except (OSError, ValueError):
        pass
    if killed.is_set():
        return EXIT_WATCHDOG
    if status is not None:
        return status
    return rc if rc >= 0 else 128 - rc


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(P: int, K: int, seconds: float) -> dict:
    """The repo's numpy restatement of the reference idiom w = w + a*(x - w)
    (oracle.sequential_mix == TF2 consensus_v3.py:153-155), single-threaded (numpy elementwise
    ufuncs use one core), on the same bucket size and neighbour count, repeated for a bounded
    sample of about `seconds` of CPU work."""
    import numpy as np
    from oracle.cfa_oracle import sequential_mix

    rng = np.random.default_rng(20261015)
    local = rng.standard_normal(P, dtype=np.float32)
    nbrs = [rng.standard_normal(P, dtype=np.float32) for _ in range(K)]
    alphas = [1.0 / (K + 1)] * K
    reps, t0 = 0, time.perf_counter()
    while True:
        sequential_mix(local, nbrs, alphas)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 1000:
            break
    gbs = reps * (K + 2) * P * 4 / el / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{reps} sequential CFA mixes of {K} neighbours x {P} fp32 on 1 core "
                      f"({cpu_model()}), numpy {np.__version__}, {el:.1f} s"}


def _pool_worker(args):
    seed, P, K, seconds, barrier, q = args
    import numpy as np
    from oracle.cfa_oracle import sequential_mix
    rng = np.random.default_rng(seed)
    local = rng.standard_normal(P, dtype=np.float32)
    nbrs = [rng.standard_normal(P, dtype=np.float32) for _ in range(K)]
    alphas = [1.0 / (K + 1)] * K
    barrier.wait()
    reps, t0 = 0, time.perf_counter()
    while True:
        sequential_mix(local, nbrs, alphas)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    q.put((reps, el))


def cpu_share() -> int:
    """CPUs this process may use: its affinity set, capped by OMP_NUM_THREADS when set (a GPU
    box's share of a large host is given there; os.cpu_count() reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline_pool(P: int, K: int, D: int, seconds: float) -> dict:
    """the reference's process model (one OS process per simulated device,
    FL_CFA_CNN_tf2.py:317-319), min(D, CPU share) worker processes each running the numpy
    restatement's sequential 8 x 25M mix concurrently for a bounded time after a common start
    barrier. Aggregate GB/s = all workers' algorithmic bytes / the longest worker's time."""
    import multiprocessing as mp
    import numpy as np
    workers = min(D, cpu_share())
    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(workers), ctx.Queue()
    procs = [ctx.Process(target=_pool_worker, args=((20261015 + w, P, K, seconds, barrier, q),))
             for w in range(workers)]
    t0 = time.perf_counter()
    for pr in procs:
        pr.start()
    res = [q.get(timeout=600) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    wall = time.perf_counter() - t0
    reps = sum(r for r, _ in res)
    el = max(e for _, e in res)
    gbs = reps * (K + 2) * P * 4 / el / 1e9
    return {"value": round(gbs, 3), "unit": "GB/s", "cores": workers, "kind": "port",
            "sample": f"{workers} processes (one per simulated device, min(D={D}, CPU share "
                      f"{cpu_share()}) of os.cpu_count()={os.cpu_count()}), {reps} sequential CFA mixes of "
                      f"{K} x {P} fp32 in {el:.1f} s ({cpu_model()}), numpy {np.__version__}, "
                      f"{wall:.1f} s wall incl. start-up"}


def load_traffic(path: str, P: int, K: int, kernel: str = None, devices_per_launch: int = 1):
    """Per-launch HBM bytes of the timed kernel from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py), if they were taken on this exact configuration."""
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None
    if (t.get("kernel") == (kernel or KERNEL) and t.get("params") == P and t.get("neighbours") == K
            and t.get("devices_per_launch", 1) == devices_per_launch):
        return t.get("hbm_bytes_per_launch")
    return None


def live_traffic(P: int, K: int, timeout: float = 150.0, ring: int = 0):
    """HBM bytes per launch of the dominant kernel, measured in THIS run: two rocprofv3 PMC passes
    (FETCH_SIZE, then WRITE_SIZE: they do not fit one TCC pass) over a child process that
    launches the same kernel on the same bucket shape (tools/pmc_probe.py), corrected as
    MI355X_MICROARCH.md prescribes (KiB; gfx950 FETCH_SIZE counts half of a wide coalesced
    read). ``ring`` = D: the probe runs the population round (D ring-window mixes) instead of
    repeated mixes of one device, i.e. the N > 1 rank's shape, where the window's rows can be
    re-read from the Infinity Cache. Returns (bytes, note) or (None, reason) when the profiler is
    unavailable."""
    import glob
    import shutil
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import per_dispatch
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not on PATH"
    vals = {}
    with tempfile.TemporaryDirectory(prefix="cfa_pmc_") as d:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = [prof, "--pmc", counter, "-d", os.path.join(d, counter), "-o", "pmc", "--output-format", "csv",
                   "--", sys.executable, os.path.join(ROOT, "tools", "pmc_probe.py"), "--params", str(P),
                   "--neighbours", str(K)] + (["--ring", str(ring)] if ring else [])
            try:
                r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=timeout)
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 {counter} pass timed out"
            files = glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True)
            if r.returncode != 0 or not files:
                return None, f"rocprofv3 {counter} pass failed (rc {r.returncode})"
            per = per_dispatch(files[0], counter, KERNEL)
            if not per:
                return None, f"no {KERNEL} dispatch in the {counter} pass"
            vals[counter] = statistics.median(per)
    read = 2.0 * vals["FETCH_SIZE"] * 1024.0
    write = vals["WRITE_SIZE"] * 1024.0
    return read + write, ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes in this run (tools/pmc_probe.py"
                          + (f" --ring {ring}: a population round of {ring} ring-window mixes" if ring else "")
                          + ", median over the launches), read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB")


class TransportError(RuntimeError):
    pass


def agree_all(ok: bool) -> bool:
    """True when ``ok`` holds on every rank (MIN over the gloo control group; local at N = 1)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return bool(ok)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return int(flag.item()) == 1


def open_transport(kind, rank, world, device, allow_fallback=False):
    """The requested transport, opened collectively: every rank takes the same decision (MIN over
    the gloo control group), so no rank is left waiting. If it cannot be opened the bench fails
    (TransportError on every rank) unless ``allow_fallback``: then torch.distributed P2P over an
    nccl (= RCCL) group, then over the gloo group (host-staged). Returns (transport, comparable):
    a line is comparable only on a device-direct transport that was opened as requested (RCCL, or
    ``--transport torch`` on an nccl group); ``--transport torch`` on the default gloo group stages
    every exchange through host memory and is marked non-comparable, named ``torch-gloo``."""
    import torch.distributed as dist
    from federated_amd.dist import TorchTransport, make_transport
    import torch

    def agree(ok: int) -> bool:
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return int(flag.item()) == 1

    t, ok, err = None, 1, ""
    try:
        t = make_transport(kind, rank, world, device)
    except Exception as exc:
        ok, err = 0, str(exc)
        print(f"[bench rank {rank}] {kind} transport failed ({exc})", file=sys.stderr)
    if agree(ok):
        staged = bool(getattr(t, "host_staged", False))
        if staged and t.name == "torch":
            t.name = "torch-gloo"
        return t, not staged
    if t is not None:
        t.close()
    if not allow_fallback:
        raise TransportError(f"the {kind} transport could not be opened on every rank"
                             + (f" (this rank: {err})" if err else "") + "; rerun with --allow-fallback "
                             "to measure on a torch.distributed transport (not comparable)")
    ok, group = 1, None
    try:
        group = dist.new_group(backend="nccl")
        probe = torch.ones(1, device=torch.device("cuda", device))
        dist.all_reduce(probe, group=group)
        torch.cuda.synchronize()
        ok = int(float(probe.item()) == float(world))
    except Exception as exc:
        ok = 0
        print(f"[bench rank {rank}] torch nccl group failed ({exc}); using gloo", file=sys.stderr)
    if agree(ok):
        t = TorchTransport(group)
        t.name = "torch-nccl"
        return t, False
    t = TorchTransport()
    t.name = "torch-gloo"
    return t, False


def seed_shard(shard, info, P):
    """Synthetic models: device g's whole bucket is seeded with 20261015 + g (the same values
    for every N and partition); a rank keeps its element slice."""
    import torch
    lo, hi = info["slice"]
    gen = torch.Generator(device=shard.device)
    full = torch.empty(P, dtype=torch.float32, device=shard.device) if (lo, hi) != (0, P) else None
    for i in range(shard.plan.L):
        gen.manual_seed(20261015 + shard.plan.first + i)
        if full is None:
            shard.models[i].normal_(generator=gen)
        else:
            full.normal_(generator=gen)
            shard.models[i].copy_(full[lo:hi])
    del full


def comm_stream():
    """The run's one exchange stream on the current device (headline, decomposition, legs, link
    probe): ``federated_amd.streams``, the rank's stream budget."""
    from federated_amd.streams import role_stream
    return role_stream("comm")


def run_leg(args, shard, world, steps, warmup, timed_kernel=True):
    """Warmup, then EXACTLY ``steps`` rounds bracketed by barrier + synchronize; returns
    (max-over-ranks seconds, per-launch kernel durations in ms)."""
    import torch
    import torch.distributed as dist

    compute = torch.cuda.current_stream()
    comm = comm_stream() if shard.plan.world > 1 else None
    interior = shard.interior_order()
    if not interior:
        timed_kernel = False
    first_i, last_i = (interior[0], interior[-1]) if interior else (None, None)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    step_idx = [0]

    # Dominant-kernel timing, live in the timed region: one HIP event pair per step around the
    # back-to-back interior mixes on the stream they run on (no events between launches, so
    # the measurement does not perturb the round); avg launch = batch time / launches. This
    # includes the sub-microsecond kernel boundaries, so it is a conservative (upper) bound on
    # the kernel duration that rocprofv3 reports.
    def timer(i, start):
        if start and i == first_i:
            ev[step_idx[0]][0].record(compute)
        elif not start and i == last_i:
            ev[step_idx[0]][1].record(compute)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(warmup):
        shard.round(compute, comm)
    barrier()
    t0 = time.perf_counter()
    for s in range(steps):
        step_idx[0] = s
        shard.round(compute, comm, timer if timed_kernel else None)
    barrier()
    elapsed = time.perf_counter() - t0
    launches = max(1, len(shard.window_passes(interior)) if args.window_batch else len(interior))
    durations = [a.elapsed_time(b) / launches for a, b in ev] if timed_kernel else []
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, durations, launches


INFINITY_CACHE_BYTES = 256 * 2**20  # MI355X_MICROARCH.md: Infinity Cache (L3) 256 MiB


def window_fits_cache(slice_P: int, K: int) -> bool:
    """Does one mix's ring window ((K + 1) input rows of ``slice_P`` fp32) fit the Infinity Cache?
    Then consecutive mixes, which share K of those rows, can re-read them from it, and an
    algorithmic-byte rate is partly cache-served (not an HBM fraction)."""
    return (K + 1) * slice_P * 4 <= INFINITY_CACHE_BYTES


def leg_slice_P(partition: str, groups, world: int, P: int) -> int:
    """A rank's row length on a partition (the slices are 64-aligned, within 64 of this)."""
    if partition == "params":
        return -(-P // world)
    if partition == "hybrid":
        return -(-P // (world // groups))
    return P


def decomposition_estimate(step_s: float, steps: int, warmup: int) -> float:
    """Seconds the two decomposition sub-legs are expected to take: each at most a headline round
    per round (the exchange alone and the mixes alone are each shorter than the overlapped
    round), warm-up included, with a 1.5x margin and the barriers' few seconds."""
    return 1.5 * 2.0 * step_s * (steps + warmup) + 5.0


def decompose_round(shard, world: int, steps: int, warmup: int, head_avg_ms: float, rates=None,
                    host_staged: bool = False, message_us: float = 0.0) -> dict:
    """The N > 1 headline round taken apart on the headline's own shard (round-4 review):

    (a) exchange only: the routed halo with no mixes, ``steps`` rounds after ``warmup``, each group
        bracketed by HIP events on the comm stream (host clock on a host-staged transport); per
        group its time (median over rounds, max over ranks), the busiest link's bytes and the rate
        that gives (GB/s per link direction), and the time the link probe's rates predict for it;
    (b) compute only: every device's mix with the halo rows already landed, HIP events around each
        round's mixes: t_mix per device, and delta = the headline's interior per-launch time (mixes
        overlapped with the exchange) / t_mix - 1, the CU and HBM time RCCL's copies take;
    (c) the model: ``predict_round_ms`` (exchange groups back to back, mixes stretched by 1 + delta
        while the exchange runs, each boundary set after its group) and the simple bound
        max(L t_mix (1 + delta), exchange + tail mixes), both max over ranks, next to the achieved
        ms per round.
    Collective over the default group. Returns the line's ``decomposition`` object."""
    import torch
    import torch.distributed as dist
    from federated_amd.population import predict_round_ms

    plan = shard.route_plan
    routed = shard.routed()
    G = len(plan.groups)
    compute = torch.cuda.current_stream()
    comm = comm_stream()

    def barrier():
        torch.cuda.synchronize()
        dist.barrier()

    marks, lane_marks = [], []
    lane = routed.lane

    def exchange_round(record: bool):
        if not host_staged:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(G + 1)]
            evs[0].record(comm)
            e0 = evs[0]
            routed.run(comm, group_done=lambda g: evs[g + 1].record(comm), lane_timing=lane is not None)
            routed.finish_lane()  # the pump has enqueued the round's H2D side (and its timing events)
        else:
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(comm)
            evs = [time.perf_counter()]

            def done(g):
                torch.cuda.synchronize()
                evs.append(time.perf_counter())
            routed.run(comm, group_done=done, lane_timing=lane is not None)
            routed.finish_lane()
        if record:
            marks.append(evs)
            if lane is not None:
                lane_marks.append((e0, lane.last_timing))

    comm.wait_stream(compute)
    for _ in range(warmup):
        exchange_round(False)
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        exchange_round(True)
    barrier()
    x_el = time.perf_counter() - t0
    if host_staged:
        per = [[(m[g + 1] - m[g]) * 1e3 for g in range(G)] for m in marks]
    else:
        per = [[m[g].elapsed_time(m[g + 1]) for g in range(G)] for m in marks]
    group_ms = [statistics.median(col) for col in zip(*per)] if G else []
    # the host lane (its own streams): when each group's lane pieces landed and when its copies
    # ended, from the exchange's start (HIP events; medians over the rounds)
    lane_arr, lane_end, lane_in, lane_out = {}, 0.0, 0.0, 0.0
    if lane_marks:
        arr = {}
        ends, ins, outs = [], [], []
        for e0, lt in lane_marks:
            for g, e in lt["groups"].items():
                arr.setdefault(g, []).append(e0.elapsed_time(e))
            ends.append(max(e0.elapsed_time(lt["i1"]), e0.elapsed_time(lt["o1"])))
            ins.append(lt["i0"].elapsed_time(lt["i1"]))
            outs.append(lt["o0"].elapsed_time(lt["o1"]))
        lane_arr = {g: statistics.median(v) for g, v in arr.items()}
        lane_end, lane_in, lane_out = statistics.median(ends), statistics.median(ins), statistics.median(outs)

    L = shard.plan.L
    evc = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for _ in range(warmup):
        shard.compute_round(compute)
    barrier()
    t0 = time.perf_counter()
    for a, b in evc:
        a.record(compute)
        shard.compute_round(compute)
        b.record(compute)
    barrier()
    c_el = time.perf_counter() - t0
    t_mix = statistics.median(a.elapsed_time(b) for a, b in evc) / max(1, L)
    delta = head_avg_ms / t_mix - 1.0 if (head_avg_ms and t_mix > 0) else 0.0

    schedule = shard.boundary_schedule()
    lane_ready = None
    if lane_arr:
        lane_ready = []
        for stage, _ in shard.stage_sets():
            pos = plan.stages.index(stage)
            got = [t for g, t in lane_arr.items() if g <= pos]
            lane_ready.append(max(got) if got else None)
    n_int = len(shard.interior_order())
    sim = predict_round_ms(group_ms, schedule, n_int, t_mix, max(0.0, delta), lane_ready, lane_end)
    x_round = max(sum(group_ms), lane_end)
    tail_devices = sum(n for g, n in schedule if g >= G - 1)
    compute_bound = L * t_mix * (1.0 + max(0.0, delta))
    simple = max(compute_bound, x_round + tail_devices * t_mix)
    # max over ranks of every figure (the round ends with the slowest rank)
    vec = torch.tensor([x_el, c_el, t_mix, delta, sim, simple, compute_bound, lane_end, lane_in, lane_out] + group_ms,
                       dtype=torch.float64)
    dist.all_reduce(vec, op=dist.ReduceOp.MAX)
    x_el, c_el, t_mix, delta, sim, simple, compute_bound, lane_end, lane_in, lane_out = vec[:10].tolist()
    group_ms = vec[10:].tolist()
    x_round = sum(group_ms)
    pred = plan.predicted_group_ms(rates, message_us=message_us) if rates else [None] * G
    groups = []
    for g in range(G):
        busiest = max(plan.group_link_elems(g, lane=False).values(), default=0) * 4
        groups.append({"ms": round(group_ms[g], 4), "busiest_link_MB": round(busiest / 1e6, 2),
                       "link_GBps": round(busiest / (group_ms[g] * 1e-3) / 1e9, 2) if group_ms[g] > 0 else None,
                       "predicted_ms": round(pred[g], 4) if pred[g] is not None else None})
    crit = sum(max(plan.group_link_elems(g, lane=False).values(), default=0) for g in range(G)) * 4
    lane_rep = None
    if lane is not None:
        from federated_amd.halo import LANE_IN, LANE_OUT
        lane_bytes = plan.lane_elems() * 4
        in_b = max((n for l, n in plan.link_elems.items() if l[0] == LANE_IN), default=0) * 4
        out_b = max((n for l, n in plan.link_elems.items() if l[1] == LANE_OUT), default=0) * 4
        pr = None
        if rates:
            rin = [r for l, r in rates.items() if l[0] == LANE_IN]
            rout = [r for l, r in rates.items() if l[1] == LANE_OUT]
            if rin and rout:
                pr = max(in_b / (min(rin) * 1e9), out_b / (min(rout) * 1e9)) * 1e3
        lane_rep = {"MB_total": round(lane_bytes / 1e6, 1), "busiest_in_MB": round(in_b / 1e6, 1),
                    "busiest_out_MB": round(out_b / 1e6, 1), "in_ms": round(lane_in, 4), "out_ms": round(lane_out, 4),
                    "end_ms": round(lane_end, 4),
                    "in_GBps": round(in_b / (lane_in * 1e-3) / 1e9, 2) if lane_in > 0 else None,
                    "out_GBps": round(out_b / (lane_out * 1e-3) / 1e9, 2) if lane_out > 0 else None,
                    "predicted_ms": round(pr, 4) if pr is not None else None,
                    "timing": "HIP events on the lane's out / in streams, from the exchange's start"}
    return {
        "host_lane": lane_rep,
        "steps": steps,
        "exchange_only_ms": round(x_el / steps * 1e3, 4),
        "exchange_groups_ms_sum": round(x_round, 4),
        "exchange_link_GBps": round(crit / (x_round * 1e-3) / 1e9, 2) if x_round > 0 else None,
        "exchange_predicted_ms": round(sum(pred), 4) if rates else None,
        "exchange_groups": groups,
        "compute_only_ms": round(c_el / steps * 1e3, 4),
        "t_mix_ms": round(t_mix, 5),
        "delta": round(delta, 4),
        "interior_devices": n_int,
        "tail_devices": tail_devices,
        "tail_ms": round(tail_devices * t_mix, 4),
        "compute_bound_ms": round(compute_bound, 4),
        "model_prediction_ms": round(simple, 4),
        "model_simulated_ms": round(sim, 4),
        "bound": "exchange" if max(x_round, lane_end) + tail_devices * t_mix > compute_bound else "compute",
        "timing": "host clock per group (host-staged transport)" if host_staged else
                  "HIP events per exchange group on the comm stream; per-round mixes on the compute stream",
    }


def lane_reserve_elems(world: int, devices: int, hl: int, hr: int, P: int, partition: str = "devices",
                       dev_groups=None) -> int:
    """The most elements the headline's route can put on the host lane for one (sender,
    receiver) pair: the pair's whole halo demand (every plan's lane share is at most that). The lane
    probe reserves and pins segments of this size, so a /dev/shm or pinning limit that would fail
    the headline's lane fails the probe (and the lane is left out of the plan) instead."""
    from federated_amd.halo import ring_transfers
    from federated_amd.population import partition_shape, slice_bounds
    gd, gp = partition_shape(partition, world, devices, dev_groups)
    if gd < 2:
        return 0
    bounds = slice_bounds(P, gp)
    demand = {}
    for t in ring_transfers(gd, devices // gd, hl, hr, P, slice_world=gp, slice_bounds=bounds):
        demand[(t.src, t.dst)] = demand.get((t.src, t.dst), 0) + (t.hi - t.lo)
    return max(demand.values(), default=0)


def headline_with_lane_fallback(measure, agree, lane: dict, probe: dict):
    """N > 1: measure the exchanging headline (``measure()``, collective). If it fails on any rank
    while the host lane was offered to its route (opening the lane, a lane wait that timed out, or
    anything else in the build and its timed rounds), the lane's pseudo-links are dropped from
    ``probe["plan_rates"]``, ``lane["error"]`` says why, and the same partition is measured again
    without the lane: the ``devices`` headline is never lost to an optional path. Returns
    (measure()'s result, None) or (None, the error) when the headline failed without the lane too
    (the caller then falls back to ``params``). ``agree(ok)``: the control plane's all-ranks AND."""
    from federated_amd.halo import is_lane_link

    def attempt():
        try:
            return measure(), None
        except Exception as exc:
            return None, f"{type(exc).__name__}: {exc}"
    res, err = attempt()
    if agree(err is None):
        return res, None
    rates = probe.get("plan_rates") or {}
    if not any(is_lane_link(l) for l in rates):
        return None, err or "the headline failed on another rank"
    lane["error"] = f"the headline with the host lane failed ({err or 'on another rank'}); measured without the lane"
    probe["plan_rates"] = {l: r for l, r in rates.items() if not is_lane_link(l)}
    res, err = attempt()
    if agree(err is None):
        return res, None
    return None, err or "the headline failed on another rank"


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the ranks are this script's children (torch.distributed.run), started before anything
        # here touches the GPU; this process only relays their line and status
        sys.exit(self_launch(sys.argv[1:], args.gpus, args.total_seconds))
    t0 = monotonic_origin(run_origin())
    budget = Budget(args.total_seconds, t0)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    wd = args.watchdog_seconds
    if wd is None:
        wd = args.total_seconds + 90.0 if args.total_seconds > 0 else 900.0
    watchdog = Watchdog(wd, rank, t0)
    rccl_log = setup_rccl_diagnostics(rank) if world > 1 else None  # before anything opens RCCL
    route_tune = "none" if args.no_autotune else args.route_tune
    if args.p2p_channels:
        os.environ["NCCL_NCHANNELS_PER_PEER"] = str(args.p2p_channels)
    import torch
    import torch.distributed as dist

    if world != args.gpus:
        print(f"[bench rank {rank}] note: --gpus {args.gpus} but WORLD_SIZE {world}; measuring {world} ranks",
              file=sys.stderr, flush=True)
    ndev = torch.cuda.device_count()
    if ndev < 1:
        sys.exit("bench.py needs a ROCm GPU")
    device = local_rank % ndev  # one rank per GPU; more ranks than GPUs only for rehearsal (torch transport)
    torch.cuda.set_device(device)
    if world > 1:
        import datetime
        # bounded control-plane waits: a peer that never arrives fails the barrier instead of
        # holding every rank for torch's 30-minute default
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=max(60.0, wd)))

    from federated_amd.engine import get_engine
    from federated_amd.population import make_ring_shard, scattered_order
    from federated_amd.streams import budget as stream_budget

    P, K = args.params, args.neighbours
    if K % 2:
        sys.exit("--neighbours must be even (ring window K/2 per side)")
    weak = args.devices_per_gpu is not None
    D = args.devices_per_gpu * world if weak else args.devices
    headline = args.partition
    eng = get_engine(device)

    # The transport (RCCL) carries the halo of the device-sharded partitions. It is opened
    # collectively before the headline (every rank takes the same decision). If it cannot be
    # opened, the headline falls back to the params partition, which exchanges nothing, the line
    # says so (config.headline_fallback) and the run exits 3; every leg that exchanges reports the
    # error in the line. Never a silent substitute transport (--allow-fallback: torch.distributed,
    # marked non-comparable).
    tstate = {"transport": None, "comparable": True, "error": None}

    def ensure_transport():
        if world == 1 or tstate["transport"] is not None or tstate["error"] is not None:
            return tstate["transport"]
        watchdog.enter("open transport")
        try:
            tstate["transport"], tstate["comparable"] = open_transport(args.transport, rank, world, device,
                                                                       args.allow_fallback)
        except TransportError as exc:
            tail = rccl_log_tail(rccl_log)
            tstate["error"] = str(exc) + (f" [RCCL log: {tail}]" if tail else "")
            if tail:
                print(f"[bench rank {rank}] RCCL log tail:\n{tail}", file=sys.stderr, flush=True)
        return tstate["transport"]

    headline_fallback = None
    headline_exchanges = world > 1 and (headline != "params" or weak)
    if headline_exchanges and ensure_transport() is None:
        print(f"[bench rank {rank}] {tstate['error']}", file=sys.stderr, flush=True)
        if weak:
            print(f"[bench rank {rank}] FATAL: the weak-scaling headline needs the transport",
                  file=sys.stderr, flush=True)
            if rank == 0:
                record_status(EXIT_TRANSPORT)
            dist.barrier()
            dist.destroy_process_group()
            sys.exit(EXIT_TRANSPORT)
        headline_fallback = {"wanted": headline, "measured": "params", "error": tstate["error"]}
        headline, headline_exchanges = "params", False

    # Per-link rates of the node, measured over the headline's transport before any route is
    # planned (federated_amd/linkprobe.py): with --route-tune links (default) they become the
    # route plan's link costs, and every line at N > 1 reports them (config.links)
    probe = {"result": None, "plan_rates": None, "message_us": 0.0, "summary": None, "error": None}
    if headline_exchanges and args.link_probe_mb > 0 and tstate["transport"] is not None:
        watchdog.enter("link probe")
        from federated_amd.linkprobe import probe_links, summarize
        t_probe = time.perf_counter()
        try:
            res = probe_links(tstate["transport"], rank, world, device, elems=int(args.link_probe_mb * 1e6 / 4))
            probe.update(result=res, summary=summarize(res, world))
            if route_tune == "links":
                probe["plan_rates"] = res["rates"]  # the route plan's input (population.make_ring_shard)
                probe["message_us"] = max(0.0, (probe["summary"].get("pieces") or {}).get("per_message_us_median")
                                          or 0.0)
        except Exception as exc:
            tail = rccl_log_tail(rccl_log)
            probe["error"] = f"{type(exc).__name__}: {exc}" + (f" [RCCL log: {tail}]" if tail else "")
            print(f"[bench rank {rank}] link probe failed: {probe['error']}", file=sys.stderr, flush=True)
        if not agree_all(probe["error"] is None):
            probe.update(result=None, plan_rates=None, summary=None, error=probe["error"] or "failed on another rank")
        if probe["summary"] is not None:
            probe["summary"]["wall_s"] = round(time.perf_counter() - t_probe, 2)

    # The host lane (federated_amd/hostlane.py): with --route-tune links, its rates with every rank
    # using it at once are measured after the links and join the plan's rates, so choose_route
    # prices every plan with and without it. A token drawn by rank 0 names the shared segments.
    lane = {"result": None, "error": None, "token": None, "opened": 0, "numa_nodes": None}
    if (headline_exchanges and args.host_lane == "auto" and probe["plan_rates"] is not None
            and args.lane_probe_mb > 0):
        watchdog.enter("host lane probe")
        from federated_amd.hostlane import new_token
        from federated_amd.linkprobe import lane_pair_rates, probe_lane
        # where every rank's GPU sits: a segment is placed on its receiver's NUMA node, and a
        # cross-node pair is priced at its own probed rate (linkprobe.lane_pair_rates)
        topo = [None] * world
        dist.all_gather_object(topo, gpu_topology(device))
        lane["topology"] = topo
        lane["numa_nodes"] = [t.get("numa_node") for t in topo]
        tok = [new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        lane["token"] = tok[0]
        t_lane = time.perf_counter()
        try:
            reserve = lane_reserve_elems(world, D, K // 2, K // 2, P, headline, args.device_groups)
        except ValueError:  # a partition the headline itself will refuse (reported there)
            reserve = 0
        try:
            # a lane whose words never arrive on this node costs one 15 s timeout, then is left out;
            # its segments are as large as the headline's plan can need, so a /dev/shm or pinning
            # limit shows here and not in the headline
            lane["result"] = probe_lane(rank, world, torch.device("cuda", device), tok[0] + "p", agree_all,
                                        elems=int(args.lane_probe_mb * 1e6 / 4), timeout_s=15.0,
                                        numa_nodes=lane["numa_nodes"], segment_elems=reserve)
        except Exception as exc:
            lane["error"] = f"{type(exc).__name__}: {exc}"
            print(f"[bench rank {rank}] host lane probe failed: {lane['error']}", file=sys.stderr, flush=True)
        if lane["result"] is not None:
            lane["result"]["wall_s"] = round(time.perf_counter() - t_lane, 2)
            probe["plan_rates"] = {**probe["plan_rates"], **lane_pair_rates(lane["result"], lane["numa_nodes"])}

    def lane_summary(xinfo=None):
        if args.host_lane == "off":
            return {"mode": "off"}
        r = lane["result"]
        if r is None and lane["error"] is None:
            return None
        out = {"error": lane["error"], "topology": lane.get("topology"), "numa_nodes": lane.get("numa_nodes"),
               "waits": "host (cfa_host_wait_word): no wait on a GPU queue"}
        if r is not None:
            out.update({"out_GBps": r["out_GBps"], "in_GBps": r["in_GBps"],
                        "message_MB": round(r["elems"] * 4 / 1e6, 1),
                        "reserved_MB_per_parity": round(r["segment_elems"] * 4 / 1e6, 1),
                        "chunk_MB": round(r["chunk_elems"] * 4 / 2**20, 2), "timing": r["timing"],
                        "wall_s": r.get("wall_s")})
        if xinfo and xinfo.get("lane"):
            out["pairs"] = xinfo["lane"].get("pairs_all")
        return out

    def build(partition, devices=None, relay=None, placement=None):
        transport = tstate["transport"]
        shard, info = make_ring_shard(rank, world, devices or D, K // 2, K // 2, P, torch.device("cuda", device),
                                      transport,
                                      eng, partition=partition, dev_groups=args.device_groups,
                                      relay=(not args.no_relay) if relay is None else relay,
                                      staged=not args.no_stages, window_batch=args.window_batch,
                                      placement_candidates=(args.placement_candidates if placement is None
                                                            else placement),
                                      placement_release=args.placement_release, link_rates=probe["plan_rates"],
                                      message_us=probe["message_us"],
                                      lane_token=f"{lane['token']}s{lane['opened']}" if lane["token"] else None,
                                      lane_agree=agree_all, lane_numa_nodes=lane["numa_nodes"])
        lane["opened"] += 1
        if world > 1 and "route_digest" in info:  # every rank must run the same schedule
            digests = [None] * world
            dist.all_gather_object(digests, info["route_digest"])
            if len(set(digests)) != 1:
                raise RuntimeError("route plans differ across ranks")
        if world > 1 and (info.get("route") or {}).get("lane"):  # every rank's pairs, for config.host_lane
            pairs = [None] * world
            mine = (info.get("lane") or {}).get("pairs") or []
            dist.all_gather_object(pairs, [dict(p, src=rank) for p in mine])
            info["lane"]["pairs_all"] = [p for part in pairs for p in (part or [])]
        seed_shard(shard, info, P)
        return shard, info

    def drop_cached():
        """Between legs: with --placement-release, return cached memory to the driver (each leg's
        calibration then settles after its scrub); by default it stays in torch's cache for the
        next leg, so no scrub runs under a timed leg."""
        if args.placement_release:
            torch.cuda.empty_cache()

    def route_choice(xshard, xinfo):
        """How the shard's route was chosen, for halo_route.autotune: with measured rates
        (--route-tune links) halo.choose_route priced the uniform, the rate-weighted and the
        direct plan at the probe's rates and kept the fastest; the chosen plan's predicted exchange
        time beside the direct-only plan's."""
        plan = xshard.route_plan
        rc = xinfo.get("route_choice") or {}
        out = {"mode": route_tune, "chosen": "relayed" if plan.relay else "direct",
               "plan": rc.get("chosen", "uniform"), "candidates_predicted_ms": rc.get("candidates"),
               "slow_links": rc.get("slow_links"), "message_us": rc.get("message_us"),
               "host_lane": xinfo.get("lane")}
        rates = probe["plan_rates"] or (probe["result"] or {}).get("rates")
        if rates:
            from federated_amd.halo import RoutePlan
            from federated_amd.hostlane import DEFAULT_CHUNK_ELEMS, first_chunk_elems
            msg = probe["message_us"]
            out["predicted_ms"] = round(plan.predicted_ms(
                rates, message_us=msg, lane_chunk_bytes=first_chunk_elems(DEFAULT_CHUNK_ELEMS) * 4), 4)
            out["direct_predicted_ms"] = round(RoutePlan(world, plan.transfers, relay=False).predicted_ms(
                rates, message_us=msg), 4)
        return out

    def build_tuned(partition, devices=None):
        """The shard of ``partition`` and how its route was chosen (N > 1): from the link probe's
        measured rates (--route-tune links, default; the plan keeps relays only where they shorten
        the predicted critical path), or round 4's wall-clock autotune (--route-tune wallclock: the
        relayed plan against the direct-only plan, a few rounds each after warm-up, max over
        ranks; the faster one is kept). Returns (shard, info, route choice or None)."""
        xshard, xinfo = build(partition, devices)
        if not (world > 1 and xinfo.get("route")):
            return xshard, xinfo, None
        if route_tune != "wallclock" or not xinfo["route"].get("relay"):
            return xshard, xinfo, route_choice(xshard, xinfo)
        tune_steps = 3
        watchdog.enter(f"route autotune ({partition})")
        t_rel, _, _ = run_leg(args, xshard, world, tune_steps, args.warmup, timed_kernel=False)
        dshard, dinfo = build(partition, devices, relay=False)
        t_dir, _, _ = run_leg(args, dshard, world, tune_steps, args.warmup, timed_kernel=False)
        tune = {"mode": "wallclock", "relayed_ms_per_step": round(t_rel / tune_steps * 1e3, 4),
                "direct_ms_per_step": round(t_dir / tune_steps * 1e3, 4)}
        # same decision on every rank: both times are maxima over ranks. The losing plan's stacks
        # stay in torch's cache: memory returned to the driver is scrubbed in the background, which
        # would slow the timed rounds (federated_amd/placement.py)
        if t_dir < t_rel:
            tune["chosen"] = "direct"
            xshard.close()  # the losing shard's lane: unpinned and unmapped
            return dshard, dinfo, tune
        dshard.close()
        del dshard
        tune["chosen"] = "relayed"
        return xshard, xinfo, tune

    def timed_scattered(xshard, steps):
        """The same rounds with the interior mixes in scattered order (consecutive mixes share no
        window rows, population.scattered_order): (max-over-ranks s, per-launch ms)."""
        xshard.mix_order = scattered_order(xshard.plan.interior(), K)
        try:
            xel, xdur, _ = run_leg(args, xshard, world, steps, args.warmup)
        finally:
            xshard.mix_order = None
        return xel, xdur

    def measure_headline(partition):
        watchdog.enter(f"build {partition} shard")
        xshard, xinfo, xtune = build_tuned(partition)
        watchdog.enter("timed rounds")
        try:
            return (xshard, xinfo, xtune) + run_leg(args, xshard, world, args.steps, args.warmup)
        except BaseException:
            xshard.close()  # a failed round: release its lane before any retry
            raise

    t_head0 = time.perf_counter()
    if world == 1:
        shard, info, autotune, elapsed, durations, launches_per_step = measure_headline(headline)
    else:
        # an exchanging headline that fails on every rank alike (an RCCL error in the first rounds
        # of a node this build never ran on) still gives a line: the params partition, which
        # exchanges nothing, then measures the headline and the run exits 3, as for a transport
        # that cannot open. (A failure on some ranks only leaves the others inside a collective;
        # the watchdog ends that run.)
        def measure_logged():
            try:
                return measure_headline(headline)
            except Exception as exc:
                tail = rccl_log_tail(rccl_log)
                print(f"[bench rank {rank}] {headline} headline failed: {type(exc).__name__}: {exc}",
                      file=sys.stderr, flush=True)
                if tail:
                    raise RuntimeError(f"{type(exc).__name__}: {exc} [RCCL log: {tail}]") from exc
                raise
        # a failure with the host lane in the plan is retried without it before any fallback
        res, err = headline_with_lane_fallback(measure_logged, agree_all, lane, probe)
        if err is not None:
            if headline == "params":
                raise RuntimeError(f"the params headline failed ({err or 'on another rank'})")
            headline_fallback = {"wanted": headline, "measured": "params",
                                 "error": err or "the headline failed on another rank"}
            headline, headline_exchanges = "params", False
            res = measure_headline("params")
        shard, info, autotune, elapsed, durations, launches_per_step = res
    # N > 1: the halo the timed rounds delivered, row by row against the rows their owners hold
    # (exact 32-bit-pattern checksums), so the line proves the exchange moved the right bytes over
    # RCCL, the relays and the host lane on this node
    halo_check = None
    if world > 1 and info.get("route") is not None:
        watchdog.enter("halo check")

        def gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
        n_rows, n_bad = shard.halo_check(gather, info["slice"][0])
        tot = torch.tensor([n_rows, n_bad], dtype=torch.int64)
        dist.all_reduce(tot)
        halo_check = {"rows": int(tot[0]), "mismatches": int(tot[1]),
                      "method": "sum of 32-bit patterns per row, receiver against owner, after the timed rounds"}
        if halo_check["mismatches"]:
            print(f"[bench rank {rank}] HALO CHECK FAILED: {n_bad} of {n_rows} halo rows differ from their owners'",
                  file=sys.stderr, flush=True)
    bytes_total = D * (K + 2) * P * 4 * args.steps  # every device's mix, all ranks (slices sum to P)
    value = bytes_total / elapsed / 1e9
    interior = shard.interior_order()
    per_launch_bytes = (K + 2) * shard.P * 4 * len(interior) // launches_per_step  # algorithmic, per launch
    avg_ms = sum(durations) / max(1, len(durations))
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    launches_timed = launches_per_step * args.steps
    route = info.get("route")
    reuse = window_fits_cache(shard_P(info, P), K)
    scat = None
    if reuse and not args.window_batch and len(interior) > 1:
        watchdog.enter("timed rounds, scattered order")
        scat = timed_scattered(shard, args.steps)
    t_headline = time.perf_counter() - t_head0

    decomp = None  # filled after the line's headline part is built (below)

    result = None
    if rank == 0:
        if weak:
            scaling = "weak"
        else:
            scaling = "strong"
        kernel = "window_vec_kernel" if args.window_batch else KERNEL
        result = {
            "metric": "device-resident GB/s, CFA reduce of K neighbour fp32 param buckets; 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded torch normal fp32 buckets, resident in HBM)",
            "config": {
                "workload": ("cfa_population_round (window passes of %d devices, rows loaded once per pass): "
                             % args.window_batch if args.window_batch else "cfa_population_round: ") +
                            "sequential CFA mix (eps=1/(K+1)) of every device of a fixed population with K "
                            "ring-window neighbours" + (", population grown with N (weak scaling)" if weak else ""),
                "params_per_bucket": P,
                "neighbours": K,
                "devices_total": D,
                "devices_per_gpu": info["devices_per_rank"],
                "partition": info["partition"],
                "headline_fallback": headline_fallback,
                "device_groups": info["device_groups"],
                "param_slices": info["param_slices"],
                "bytes_per_device_mix": (K + 2) * P * 4,
                "window_batch": args.window_batch,
                "transport": tstate["transport"].name if headline_exchanges else "none (no exchange)",
                "comparable": tstate["comparable"] if headline_exchanges else True,
                "halo_route": ({k: route[k] for k in ("relay", "lane", "stages", "groups", "messages",
                                                     "max_messages_per_rank_group", "link_cost")}
                               | {"lane_MB": round(route["lane_elems"] * 4 / 1e6, 1),
                                  "max_link_MB": round(route["max_link_elems"] * 4 / 1e6, 1),
                                  "critical_MB": round(route["critical_elems"] * 4 / 1e6, 1),
                                  "autotune": autotune,
                                  "predicted_critical_ms": (autotune or {}).get("predicted_ms"),
                                  "achieved_critical_ms": (decomp or {}).get("exchange_groups_ms_sum")})
                if route else None,
                "links": probe["summary"] if probe["error"] is None else {"error": probe["error"]},
                "halo_check": halo_check,
                "host_lane": lane_summary(info) if headline_exchanges else None,
                "placement": info.get("placement"),
                "halo_carved": info.get("halo_carved"),
                "cache_reuse": reuse,
                "gpus_visible": ndev,
                "ranks_share_gpus": world > ndev,
                "rccl_env": {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))},
                "gpu_max_hw_queues": hw_queues_report(),
                "streams": {"compute": "torch current stream",
                            "roles": {str(d): r for d, r in stream_budget().items()},
                            "waits": "none on a GPU queue (host lane: host-side waits)"},
                "rccl_version": rccl_version() if world > 1 else None,
                "parallelism": f"population-{info['partition']}{world}",
                "rows_note": (f"each rank's rows are {shard_P(info, P)} elements, so a mix's {K + 1}-row window "
                              f"({(K + 1) * shard_P(info, P) * 4 / 2**20:.0f} MiB) fits the 256 MiB Infinity Cache "
                              "and consecutive mixes can re-read the rows they share from it: value counts "
                              "algorithmic bytes, value_scattered is the same round with no two consecutive mixes "
                              "sharing a row (DESIGN.md §5)") if reuse else None,
                "budget": {"total_s": args.total_seconds, "headline_s": round(t_headline, 1)},
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kernel,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "avg_launch_ms": round(avg_ms, 5),
                "step_avg_launch_ms_median": round(statistics.median(durations), 5) if durations else None,
                "step_avg_launch_ms_min": round(min(durations), 5) if durations else None,
                "launches_timed": launches_timed,
                "bytes_per_launch": per_launch_bytes,
                "timing": "HIP events around each step's back-to-back interior mixes / launches",
                # the whole job against the aggregate HBM peak of its GPUs (north_star: GB/s at
                # 1/2/4/8 GPUs "as absolute numbers and as fraction of the HBM roofline"); at N > 1
                # this includes the exchange
                "job_peak": HBM_PEAK_GBS * world,
                "job_frac": round(value / (HBM_PEAK_GBS * world), 4),
                "cache_reuse": reuse,
                "traffic": load_traffic(
                    args.traffic_json or os.path.join(ROOT, "profiles", "r01_window_pmc_traffic.json"
                                                      if args.window_batch else "r01_pmc_traffic.json"),
                    shard_P(info, P), K, kernel, args.window_batch or 1),
            },
        }
        if scat is not None:
            xel, xdur = scat
            result["value_scattered"] = round(bytes_total / xel / 1e9, 2)
            result["ms_per_step_scattered"] = round(xel / args.steps * 1e3, 4)
            if xdur:
                xavg = sum(xdur) / len(xdur)
                rl = result["roofline"]
                rl["avg_launch_ms_scattered"] = round(xavg, 5)
                rl["achieved_scattered"] = round(per_launch_bytes / (xavg * 1e-3) / 1e9, 1)
                rl["frac_scattered"] = round(rl["achieved_scattered"] / HBM_PEAK_GBS, 4)
        pl = info.get("placement") or {}
        if pl.get("plain_us"):
            # the same mix on candidate pair (0, 0), the first allocation of each stack: what the
            # population runs at without the placement choice (probe timing, HIP events)
            rl = result["roofline"]
            plain = (K + 2) * shard_P(info, P) * 4 / (pl["plain_us"] * 1e-6) / 1e9
            rl["achieved_plain_alloc"] = round(plain, 1)
            rl["frac_plain_alloc"] = round(plain / HBM_PEAK_GBS, 4)
            rl["placement_rejected_cached_GiB"] = pl.get("rejected_cached_GiB")

    # what the report still needs after the legs: rank 0's PMC passes (a child process each) and,
    # at N = 1, the CPU baselines and the e2e leg
    live = not args.no_live_traffic and not args.window_batch
    pmc_est = 45.0
    reserve = 15.0 + (2 * pmc_est if live else 0.0)
    legs = {}
    legs_n1 = {}
    leg_failed = False

    import threading
    report_lock = threading.Lock()

    def report_partial(mark):
        """Rank 0: print the line once, with what is measured so far and ``mark(out)`` recording
        the part that did not finish (the headline is complete). Returns the exit status: 5, or 3
        after a headline fallback. The other ranks give rank 0 time to print first
        (torch.distributed.run ends every rank once one has exited)."""
        code = EXIT_TRANSPORT if headline_fallback else EXIT_LEG
        with report_lock:
            if rank == 0 and not report_partial.done:
                out = None
                for _ in range(50):  # the main thread may be adding a leg right now
                    try:
                        out = json.loads(json.dumps(result))
                        break
                    except RuntimeError:
                        time.sleep(0.01)
                if out is None:
                    out = {k: v for k, v in result.items() if k != "partitions"}
                mark(out)
                out["exit_status"] = code
                print(json.dumps(out), flush=True)
                record_status(code)
                report_partial.done = True
        if rank != 0:
            wait_for_status(15.0)
        return code
    report_partial.done = False

    # N = 1: the same rounds on placement-calibrated stacks (placement.calibrated_stacks: the fastest
    # of --placement-leg allocations per stack), beside the plain-allocation headline; the headline's
    # stacks are released first and the leg's candidates go back to the driver after it
    if world == 1 and args.placement_leg > 1 and args.placement_candidates <= 1:
        est = 2.5 * t_headline + 30.0
        if budget.left() - reserve - 45.0 >= est:
            watchdog.enter("placement-calibrated leg")
            shard.close()
            del shard
            try:
                cshard, cinfo = build(headline, placement=args.placement_leg)
                cel, cdur, claunch = run_leg(args, cshard, world, args.steps, args.warmup)
                cavg = sum(cdur) / max(1, len(cdur))
                cach = per_launch_bytes / (cavg * 1e-3) / 1e9 if cavg > 0 else 0.0
                legs_n1["placement_calibrated"] = {
                    "value": round(bytes_total / cel / 1e9, 2), "ms_per_step": round(cel / args.steps * 1e3, 4),
                    "avg_launch_ms": round(cavg, 5), "achieved": round(cach, 1),
                    "frac": round(cach / HBM_PEAK_GBS, 4), "placement": cinfo.get("placement"),
                    "note": "the headline's rounds on stacks chosen as the fastest of %d allocations each "
                            "(federated_amd/placement.py); value is the plain-allocation figure" % args.placement_leg}
                cshard.close()
                del cshard
            except Exception as exc:
                legs_n1["placement_calibrated"] = {"error": f"{type(exc).__name__}: {exc}"}
            torch.cuda.empty_cache()
        else:
            legs_n1["placement_calibrated"] = {"skipped": "budget", "estimate_s": round(est, 1)}
        if rank == 0:
            result["legs"] = legs_n1

    # N > 1: the headline round taken apart on the headline's own shard (exchange only, compute
    # only, the model's prediction), so a scaling result explains itself. Budget-gated (the
    # headline never is) and run as a leg with its own watchdog budget: if it hangs in a
    # collective, rank 0 prints the line with the headline and the decomposition's error.
    if world > 1 and headline_exchanges and route is not None and not args.no_decomposition:
        dsteps = args.decomp_steps or min(args.steps, 10)
        est = decomposition_estimate(elapsed / args.steps, dsteps, args.warmup)
        if agree_all(budget.left() - reserve >= est):
            seconds = budget.left() - reserve
            if args.leg_seconds > 0:
                seconds = min(seconds, args.leg_seconds)

            def decomp_expired(phase, seconds=seconds):
                why = f"did not finish within {seconds:.0f} s (phase '{phase}')"
                return report_partial(lambda out: out.__setitem__("decomposition", {"error": why}))
            watchdog.leg("decomposition (exchange only, compute only)", seconds, decomp_expired)
            try:
                decomp = decompose_round(shard, world, dsteps, args.warmup, avg_ms,
                                         probe["plan_rates"] or (probe["result"] or {}).get("rates"),
                                         bool(getattr(tstate["transport"], "host_staged", False)),
                                         probe["message_us"])
                decomp["achieved_ms"] = round(elapsed / args.steps * 1e3, 4)
            except Exception as exc:
                decomp = {"error": f"{type(exc).__name__}: {exc}"}
                print(f"[bench rank {rank}] decomposition failed: {decomp['error']}", file=sys.stderr, flush=True)
            if not agree_all("error" not in decomp):
                decomp = {"error": decomp.get("error", "failed on another rank")}
            watchdog.end_leg()
        else:
            decomp = {"skipped": "budget", "estimate_s": round(est, 1), "budget_left_s": round(budget.left(), 1)}
        if rank == 0:
            result["decomposition"] = decomp
            result["config"]["halo_route"]["achieved_critical_ms"] = decomp.get("exchange_groups_ms_sum")

    if world > 1 and not args.no_extra_legs and not weak:
        shard.close()
        del shard
        drop_cached()
        if rank == 0:
            result["partitions"] = legs  # filled as the legs finish (a leg over budget reports what it has)
        notes = {
            "params": "same population and steps, every rank holds a 1/N element slice of every bucket "
                      "(SURVEY §8 e (1)); no exchange",
            "devices": "same population and steps in contiguous device blocks (north_star: devices sharded); "
                       "the routed halo of the ring window exchanged every round",
            "hybrid2": "same population and steps, 2 device blocks, each split over N/2 element slices; routed "
                       "halo between ranks holding the same slice",
            "weak": f"{args.devices} devices per GPU (population grown with N), devices partition",
        }

        def report_early(name, why):
            """The line with the legs measured so far and leg ``name`` marked with ``why``."""
            return report_partial(lambda out: out.setdefault("partitions", {}).__setitem__(
                name, {"error": why, "note": notes[name]}))

        def leg_expired(name, seconds):
            # runs on the watchdog thread of a rank whose leg budget ran out (every rank's budget
            # starts at the same collective, so they expire together)
            return lambda phase: report_early(name, f"did not finish within {seconds:.0f} s (phase '{phase}')")

        for name, part, groups in extra_legs(world, D, headline, not args.no_weak_leg):
            slice_P = leg_slice_P(part, groups, world, P)
            est = leg_estimate(name, world, t_headline, scattered=window_fits_cache(slice_P, K))
            if not agree_all(budget.left() - reserve >= est):
                legs[name] = {"skipped": "budget", "estimate_s": round(est, 1),
                              "budget_left_s": round(budget.left(), 1), "note": notes[name]}
                continue
            seconds = budget.left() - reserve
            if args.leg_seconds > 0:
                seconds = min(seconds, args.leg_seconds)
            watchdog.leg(f"{name} leg", seconds, leg_expired(name, seconds))
            leg, err = {"note": notes[name]}, None
            xshard = None
            t_leg = time.perf_counter()
            try:
                if part != "params" and ensure_transport() is None:
                    raise TransportError(tstate["error"])
                watchdog.enter(f"{name} leg")
                saved, args.device_groups = args.device_groups, groups
                try:
                    if name == "weak":
                        Dw = args.devices * world
                        xshard, xinfo, xtune = build_tuned("devices", Dw)
                        leg_bytes = Dw * (K + 2) * P * 4 * args.steps
                        leg["devices_total"] = Dw
                    else:
                        xshard, xinfo, xtune = build_tuned(part)
                        leg_bytes = bytes_total
                finally:
                    args.device_groups = saved
                xel, _, _ = run_leg(args, xshard, world, args.steps, args.warmup, timed_kernel=False)
                leg.update({"value": round(leg_bytes / xel / 1e9, 2), "ms_per_step": round(xel / args.steps * 1e3, 4)})
                leg_reuse = window_fits_cache(shard_P(xinfo, P), K)
                leg["cache_reuse"] = leg_reuse
                if leg_reuse and not args.window_batch and len(xshard.plan.interior()) > 1:
                    watchdog.enter(f"{name} leg, scattered order")
                    sel, _ = timed_scattered(xshard, args.steps)
                    leg["value_scattered"] = round(leg_bytes / sel / 1e9, 2)
                    leg["ms_per_step_scattered"] = round(sel / args.steps * 1e3, 4)
                if xinfo.get("route"):
                    leg["halo_critical_MB"] = round(xinfo["route"]["critical_elems"] * 4 / 1e6, 1)
                    leg["halo_carved"] = xinfo.get("halo_carved")
                if xtune:
                    leg["autotune"] = xtune
                if xinfo.get("lane"):
                    leg["host_lane"] = xinfo["lane"]
                if part != "params":
                    leg["transport"] = tstate["transport"].name
                    leg["comparable"] = tstate["comparable"]
                leg["wall_s"] = round(time.perf_counter() - t_leg, 1)
            except Exception as exc:  # reported in the line; every rank takes the same decision below
                err = f"{type(exc).__name__}: {exc}"
                print(f"[bench rank {rank}] {name} leg failed: {err}", file=sys.stderr, flush=True)
            finally:
                if xshard is not None:
                    xshard.close()
                xshard = None
                drop_cached()
            try:
                all_ok = agree_all(err is None)
            except Exception as exc:  # a peer has left (its leg budget ran out first): report and end
                print(f"[bench rank {rank}] control plane lost a peer in the {name} leg ({exc})",
                      file=sys.stderr, flush=True)
                code = report_early(name, err or f"a rank left during the leg ({type(exc).__name__})")
                record_status(code)
                os._exit(code)
            if not all_ok:
                leg = {"error": err or "failed on another rank", "note": notes[name]}
                leg_failed = True
            legs[name] = leg
            watchdog.end_leg()
        if rank == 0 and not legs:
            result.pop("partitions", None)
    if world > 1:
        dist.barrier()
    # CPU baselines: rank 0, N = 1 only (bounded samples), each only if the budget left covers it
    watchdog.enter("baselines and report")
    skipped = []
    if rank == 0:
        e2e = args.e2e and world == 1
        e2e_est = 30.0 if e2e else 0.0
        tail = e2e_est + (2 * pmc_est if live else 0.0)
        result["cpu_baseline"] = None
        if world == 1 and not args.no_cpu_baseline:
            if budget.allows(args.cpu_seconds + 10 + tail):
                result["cpu_baseline"] = cpu_baseline(P, K, args.cpu_seconds)
            else:
                skipped.append("cpu_baseline")
            if args.cpu_pool_seconds > 0:
                if budget.allows(args.cpu_pool_seconds + 20 + tail):
                    result["cpu_baseline_pool"] = cpu_baseline_pool(P, K, D, args.cpu_pool_seconds)
                else:
                    skipped.append("cpu_baseline_pool")
        if live:
            # the dominant mix's bucket shape; on rows short enough for the Infinity Cache to re-serve
            # (rows_note), the rank's own ring round (its devices, its element slice)
            rl = result["roofline"]
            pass_s = min(150.0, (budget.left() - e2e_est - 10.0) / 2)
            if pass_s >= 30.0:
                live_b, note = live_traffic(shard_P(info, P), K, timeout=pass_s,
                                            ring=info["devices_per_rank"] if world > 1 and reuse else 0)
                if live_b is not None:
                    rl["traffic_committed"] = rl["traffic"]
                    rl["traffic"] = round(live_b, 1)
                    rl["traffic_over_algorithmic"] = round(live_b / rl["bytes_per_launch"], 5)
                rl["traffic_source"] = note if live_b is not None else f"committed profile ({note})"
            else:
                skipped.append("live_traffic")
                rl["traffic_source"] = "committed profile (live PMC passes skipped: budget)"
        if e2e:
            if budget.allows(e2e_est):
                from federated_amd.staging import measure_e2e
                result["e2e"] = measure_e2e(eng, P, K)
            else:
                skipped.append("e2e")
    if world > 1:
        # every rank's RCCL warnings (NCCL_DEBUG=WARN, setup_rccl_diagnostics) into the line, so a
        # scaling run on a node this build never ran on says what RCCL complained about
        watchdog.enter("gather RCCL logs")
        tails = [None] * world
        dist.all_gather_object(tails, rccl_log_tail(rccl_log, 600))
        if rank == 0:
            result["config"]["rccl_log"] = {str(r): t for r, t in enumerate(tails) if t} or None
    halo_bad = bool(halo_check and halo_check["mismatches"])
    code = EXIT_TRANSPORT if headline_fallback else (EXIT_LEG if (leg_failed or halo_bad) else 0)
    if rank == 0:
        result["config"]["budget"].update({"skipped": skipped, "left_s": round(budget.left(), 1)})
        result["exit_status"] = code
        print(json.dumps(result), flush=True)
        record_status(code)
    if world > 1:
        # no rank leaves before rank 0's line is out: torch.distributed.run ends every rank as soon
        # as one exits with a non-zero status
        watchdog.enter("final barrier")
        dist.barrier()
    if tstate["transport"] is not None:
        tstate["transport"].close()
    if world > 1:
        dist.destroy_process_group()
    if rccl_log and os.path.basename(rccl_log).startswith("cfa_rccl_r"):
        try:
            os.unlink(rccl_log)  # ours (setup_rccl_diagnostics), its tail is in the line
        except OSError:
            pass
    watchdog.done()
    if code:
        sys.exit(code)


def rccl_version():
    """ncclGetVersion of the RCCL libcfa runs on (e.g. 22703 = 2.27.3), or None."""
    import ctypes
    from federated_amd import _lib
    v = ctypes.c_int(0)
    try:
        _lib.call("cfa_rccl_version", ctypes.byref(v))
    except Exception:
        return None
    return int(v.value)


def gpu_topology(device: int) -> dict:
    """Where this rank's GPU sits: its PCI address, the NUMA node the kernel reports for it and the
    CPUs this process may run on (the host lane's D2H / H2D cross that path; read-only sysfs)."""
    import torch
    out = {"device": device}
    try:
        pr = torch.cuda.get_device_properties(device)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        out["pci"] = bdf
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as fh:
            out["numa_node"] = int(fh.read().strip())
    except (OSError, ValueError, AttributeError, RuntimeError):
        pass
    try:
        cpus = sorted(os.sched_getaffinity(0))
        out["cpus"] = f"{cpus[0]}-{cpus[-1]} ({len(cpus)})" if cpus else None
    except (AttributeError, OSError):
        pass
    return out


def shard_P(info, P):
    lo, hi = info["slice"]
    return hi - lo


if __name__ == "__main__":
    main()
