#!/usr/bin/env python3
"""Benchmark: device-resident CFA reduction of K neighbour fp32 buckets on MI355X.

Metric (BASELINE.json): "device-resident GB/s, CFA reduce of K neighbour fp32 param buckets;
1/2/4/8 GPU". Workload (BASELINE.json north_star target): 8 neighbour buckets x 25M fp32 params
mixed into each device's local model (the TF2 sequential CFA rule, eps = 1/(K+1),
consensus_v3.py:145,153-155), for every device of a simulated population of D = 128 devices on
a wrap-around ring window of K = 8 neighbours. One step = one consensus round of the whole
population.

Scaling (SURVEY §8 e: "Strong scaling, fixed population"): the population stays D = 128 for
every N. At N > 1 the headline ``value`` uses the element split SURVEY §8 e (1) names for the
8 x 25M bucket scaling run (``--partition params``: every rank holds a 1/N slice of every
device's bucket; elements are independent, so there is no exchange). Beside it, in
``partitions``, the same population, steps and clock on the other partitions: ``devices``
(contiguous device blocks, north_star's "devices sharded": a round is the routed halo exchange of
the 2x4 boundary buckets of each rank -- federated_amd/halo.py: direct plus relayed xGMI paths,
sent row by row -- overlapped with the interior mixes, each boundary device mixing as soon as the
rows it reads have landed), ``hybrid2`` (from N = 4: 2 device blocks x N/2 slices) and ``weak``
(128 devices per GPU, D = 128 N). ``--partition devices|hybrid`` makes either the headline;
``--devices-per-gpu L`` keeps the per-GPU population fixed instead (weak scaling, D = L*N).

Each rank's population stacks are placement-calibrated before the timed region
(``--placement-candidates``, federated_amd/placement.py: the fastest of 4 allocations per stack,
probed with the same mix; the probe is reported in ``config.placement``).

value = algorithmic bytes of all mixes on all ranks / max-over-ranks wall time, with
algorithmic bytes = (K + 2) * P * 4 per device mix (K neighbour reads + local read + output
write). Inputs are resident in HBM when the timed region starts.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU; RANK/LOCAL_RANK/WORLD_SIZE from the environment).
The transport (RCCL) is opened after the params headline, which exchanges nothing. If it cannot be
opened, every leg that exchanges reports the error in ``partitions`` (``--allow-fallback`` runs
them on a torch.distributed transport instead, marked non-comparable); with a headline that
exchanges (``--partition devices|hybrid``, weak scaling) the run exits 3. A leg that does not finish
within ``--leg-seconds`` is reported as an error and the line is printed with the legs measured so
far.
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
    p.add_argument("--partition", default=None, choices=["devices", "params", "hybrid"],
                   help="params (default at N > 1, SURVEY §8 e (1)): every rank holds a 1/N element slice "
                        "of every bucket (no exchange); devices: contiguous device blocks + routed halo "
                        "exchange; hybrid: --device-groups blocks, each split over N/groups slices")
    p.add_argument("--device-groups", type=int, default=None)
    p.add_argument("--no-relay", action="store_true", help="halo on the direct links only")
    p.add_argument("--no-stages", action="store_true",
                   help="whole halo in one exchange step (boundary devices wait for all of it)")
    p.add_argument("--no-extra-legs", "--no-params-leg", dest="no_extra_legs", action="store_true",
                   help="N > 1: skip the other partitions' measurements (devices, hybrid2) beside the headline")
    p.add_argument("--no-autotune", action="store_true",
                   help="N > 1: time the relayed route as planned, without first comparing it with "
                        "the direct-only route")
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
    p.add_argument("--placement-candidates", type=int, default=4,
                   help="allocate each population stack this many times and keep the fastest, timed "
                        "with the population's own mix before the timed region (federated_amd/placement.py; "
                        "1 = plain allocation)")
    p.add_argument("--placement-release", action="store_true",
                   help="return the rejected placement candidates to the driver (then wait out its "
                        "background scrub) instead of leaving them in torch's caching allocator")
    p.add_argument("--watchdog-seconds", type=float, default=900.0,
                   help="end the run with status 124 and the phase it was in if it has not finished "
                        "after this long (a collective that never completes; 0 = off)")
    p.add_argument("--leg-seconds", type=float, default=240.0,
                   help="N > 1: budget of each extra leg (partitions beside the headline); a leg that "
                        "has not finished by then is reported as an error in the line, which is then "
                        "printed with the legs measured so far (0 = no per-leg budget)")
    return p.parse_args()


class Watchdog:
    """Ends the process (status 124) with the phase it was stuck in if the run has not finished in
    time. A collective that never completes on one rank (a peer that died inside RCCL, a
    mismatched exchange) otherwise hangs every rank until an outer limit kills the job without
    saying where; torch.distributed.run tears the other ranks down once this one exits."""

    def __init__(self, seconds: float, rank: int):
        import threading
        self.phase, self.rank, self._done = "start-up", rank, threading.Event()
        self.t0 = time.perf_counter()
        self._leg = None  # (deadline, budget, on_expire) of a phase entered with its own budget
        self.seconds = seconds
        threading.Thread(target=self._watch, daemon=True).start()

    def _watch(self):
        while not self._done.wait(0.25):
            now = time.perf_counter()
            leg = self._leg
            if leg is not None and now > leg[0]:
                print(f"[bench rank {self.rank}] watchdog: phase '{self.phase}' did not finish within its "
                      f"{leg[1]:.0f} s budget", file=sys.stderr, flush=True)
                os._exit(leg[2](self.phase))
            if self.seconds > 0 and now - self.t0 > self.seconds:
                print(f"[bench rank {self.rank}] FATAL: watchdog: not finished after {self.seconds:.0f} s, "
                      f"stuck in phase '{self.phase}'", file=sys.stderr, flush=True)
                os._exit(124)

    def enter(self, phase: str) -> None:
        self.phase = phase

    def leg(self, phase: str, budget: float, on_expire) -> None:
        """Enter ``phase`` with a budget of its own (seconds, 0 = none) that holds until ``end_leg``
        whatever phases are entered meanwhile: if it runs out, ``on_expire(phase)`` runs on the
        watchdog thread and its return value is the exit status (the N > 1 bench's extra legs: the
        headline is already measured, so a leg stuck in a collective is reported in the line instead
        of losing the whole run)."""
        self.phase = phase
        self._leg = (time.perf_counter() + budget, budget, on_expire) if budget > 0 else None

    def end_leg(self) -> None:
        self._leg = None

    def done(self) -> None:
        self._done.set()


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


def run_leg(args, shard, world, steps, warmup, timed_kernel=True):
    """Warmup, then EXACTLY ``steps`` rounds bracketed by barrier + synchronize; returns
    (max-over-ranks seconds, per-launch kernel durations in ms)."""
    import torch
    import torch.distributed as dist

    compute = torch.cuda.current_stream()
    comm = torch.cuda.Stream() if shard.plan.world > 1 else None
    interior = shard.plan.interior()
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


def main():
    args = parse()
    watchdog = Watchdog(args.watchdog_seconds, int(os.environ.get("RANK", "0")))
    if args.p2p_channels:
        os.environ["NCCL_NCHANNELS_PER_PEER"] = str(args.p2p_channels)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
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
                                timeout=datetime.timedelta(seconds=max(60.0, args.watchdog_seconds)))

    from federated_amd.engine import get_engine
    from federated_amd.population import make_ring_shard

    P, K = args.params, args.neighbours
    if K % 2:
        sys.exit("--neighbours must be even (ring window K/2 per side)")
    weak = args.devices_per_gpu is not None
    D = args.devices_per_gpu * world if weak else args.devices
    if args.partition is None:
        # SURVEY §8 e (1): "within one bucket elements are independent => split P across G GPUs with
        # no exchange. Used for the '8 x 25M bucket' scaling run"; the device-sharded population
        # (with its halo exchange) is measured beside it (partitions.devices)
        args.partition = "params" if world > 1 and not weak else "devices"
    eng = get_engine(device)

    # The transport (RCCL) carries the halo of the device-sharded partitions only. The params
    # headline (every rank a 1/N element slice, no exchange) needs none, so at N > 1 it is measured
    # first and the transport is opened after it, for the legs that exchange. A transport that cannot
    # be opened then fails those legs (an "error" entry in the line, never a silent fallback); with
    # a headline that needs it (--partition devices|hybrid, or weak scaling) the run exits 3.
    tstate = {"transport": None, "comparable": True, "error": None}

    def ensure_transport():
        if world == 1 or tstate["transport"] is not None or tstate["error"] is not None:
            return tstate["transport"]
        watchdog.enter("open transport")
        try:
            tstate["transport"], tstate["comparable"] = open_transport(args.transport, rank, world, device,
                                                                       args.allow_fallback)
        except TransportError as exc:
            tstate["error"] = str(exc)
        return tstate["transport"]

    headline_exchanges = world > 1 and (args.partition != "params" or weak)
    if headline_exchanges and ensure_transport() is None:
        print(f"[bench rank {rank}] FATAL: {tstate['error']}", file=sys.stderr, flush=True)
        dist.destroy_process_group()
        sys.exit(3)

    def build(partition, devices=None, relay=None):
        transport = tstate["transport"]
        shard, info = make_ring_shard(rank, world, devices or D, K // 2, K // 2, P, torch.device("cuda", device),
                                      transport,
                                      eng, partition=partition, dev_groups=args.device_groups,
                                      relay=(not args.no_relay) if relay is None else relay,
                                      staged=not args.no_stages, window_batch=args.window_batch,
                                      placement_candidates=args.placement_candidates,
                                      placement_release=args.placement_release)
        if world > 1 and "route_digest" in info:  # every rank must run the same schedule
            digests = [None] * world
            dist.all_gather_object(digests, info["route_digest"])
            if len(set(digests)) != 1:
                raise RuntimeError("route plans differ across ranks")
        seed_shard(shard, info, P)
        return shard, info

    watchdog.enter(f"build {args.partition} shard")
    def drop_cached():
        """Between legs: with --placement-release, return cached memory to the driver (each leg's
        calibration then settles after its scrub); by default it stays in torch's cache for the
        next leg, so no scrub runs under a timed leg."""
        if args.placement_release:
            torch.cuda.empty_cache()

    def build_tuned(partition, devices=None):
        """The shard of ``partition``; with a relayed route at N > 1, route autotune before any timed
        region: the relayed plan against the direct-only plan, a few rounds each after warm-up, max
        over ranks; the faster one is kept (the cost model assumes every link runs at the same
        rate; this checks it on the node). Returns (shard, info, autotune or None)."""
        xshard, xinfo = build(partition, devices)
        if not (world > 1 and xinfo.get("route", {}).get("relay") and not args.no_autotune):
            return xshard, xinfo, None
        tune_steps = 3
        watchdog.enter(f"route autotune ({partition})")
        t_rel, _, _ = run_leg(args, xshard, world, tune_steps, args.warmup, timed_kernel=False)
        dshard, dinfo = build(partition, devices, relay=False)
        t_dir, _, _ = run_leg(args, dshard, world, tune_steps, args.warmup, timed_kernel=False)
        tune = {"relayed_ms_per_step": round(t_rel / tune_steps * 1e3, 4),
                "direct_ms_per_step": round(t_dir / tune_steps * 1e3, 4)}
        # same decision on every rank: both times are maxima over ranks. The losing plan's stacks
        # stay in torch's cache: memory returned to the driver is scrubbed in the background, which
        # would slow the timed rounds (federated_amd/placement.py)
        if t_dir < t_rel:
            tune["chosen"] = "direct"
            return dshard, dinfo, tune
        del dshard
        tune["chosen"] = "relayed"
        return xshard, xinfo, tune

    shard, info, autotune = build_tuned(args.partition)
    watchdog.enter("timed rounds")
    elapsed, durations, launches_per_step = run_leg(args, shard, world, args.steps, args.warmup)
    bytes_total = D * (K + 2) * P * 4 * args.steps  # every device's mix, all ranks (slices sum to P)
    value = bytes_total / elapsed / 1e9
    interior = shard.plan.interior()
    per_launch_bytes = (K + 2) * shard.P * 4 * len(interior) // launches_per_step  # algorithmic, per launch
    avg_ms = sum(durations) / max(1, len(durations))
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    launches_timed = launches_per_step * args.steps
    route = info.get("route")

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
                "device_groups": info["device_groups"],
                "param_slices": info["param_slices"],
                "bytes_per_device_mix": (K + 2) * P * 4,
                "window_batch": args.window_batch,
                "transport": tstate["transport"].name if headline_exchanges else "none (no exchange)",
                "comparable": tstate["comparable"] if headline_exchanges else True,
                "halo_route": ({k: route[k] for k in ("relay", "stages", "groups", "messages",
                                                     "max_messages_per_rank_group")}
                               | {"max_link_MB": round(route["max_link_elems"] * 4 / 1e6, 1),
                                  "critical_MB": round(route["critical_elems"] * 4 / 1e6, 1),
                                  "autotune": autotune}) if route else None,
                "placement": info.get("placement"),
                "halo_carved": info.get("halo_carved"),
                "rccl_env": {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))},
                "rccl_version": rccl_version() if world > 1 else None,
                "parallelism": f"population-{info['partition']}{world}",
                "rows_note": (f"each rank's rows are {shard_P(info, P)} elements; below about 6M elements the "
                              "ring window's 9 rows fit the 256 MB Infinity Cache, so a mix can re-read the 8 rows "
                              "it shares with the previous device's mix from it (DESIGN.md §5); value counts "
                              "algorithmic bytes, and roofline.traffic (L2 misses, FETCH_SIZE / WRITE_SIZE) counts "
                              "reads the Infinity Cache serves as well") if world > 1 and info["partition"] == "params" else None,
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
                "traffic": load_traffic(
                    args.traffic_json or os.path.join(ROOT, "profiles", "r01_window_pmc_traffic.json"
                                                      if args.window_batch else "r01_pmc_traffic.json"),
                    shard_P(info, P), K, kernel, args.window_batch or 1),
            },
        }
        pl = info.get("placement") or {}
        if pl.get("plain_us"):
            # the same mix on candidate pair (0, 0), the first allocation of each stack: what the
            # population runs at without the placement choice (probe timing, HIP events)
            rl = result["roofline"]
            plain = (K + 2) * shard_P(info, P) * 4 / (pl["plain_us"] * 1e-6) / 1e9
            rl["achieved_plain_alloc"] = round(plain, 1)
            rl["frac_plain_alloc"] = round(plain / HBM_PEAK_GBS, 4)
            rl["placement_rejected_cached_GiB"] = pl.get("rejected_cached_GiB")
    legs = {}
    if rank == 0 and world > 1 and not args.no_extra_legs and not weak:
        result["partitions"] = legs  # filled as the legs finish (a leg over budget reports what it has)
    if world > 1 and not args.no_extra_legs and not weak:
        del shard
        drop_cached()
        notes = {
            "params": "same population and steps, every rank holds a 1/N element slice of every bucket "
                      "(SURVEY §8 e (1)); no exchange",
            "devices": "same population and steps in contiguous device blocks (north_star: devices sharded); "
                       "the routed halo of the ring window exchanged every round",
            "hybrid": "same population and steps, 2 device blocks, each split over N/2 element slices; routed "
                      "halo between ranks holding the same slice",
            "weak": f"{args.devices} devices per GPU (population grown with N), devices partition",
        }
        extra = [(part, None) for part in ("params", "devices") if part != args.partition]
        if world >= 4 and D % 2 == 0 and args.partition != "hybrid":
            extra.append(("hybrid", 2))
        if not args.no_weak_leg:
            # weak form for reference: the single-GPU population on every rank (D = 128 N) in device
            # blocks, the routed halo hidden under 120 interior mixes per rank
            extra.append(("weak", None))

        import threading
        report_lock = threading.Lock()

        def report_early(name, why):
            """Rank 0: print the line once, with the legs measured so far and ``name`` marked with
            ``why`` (the headline is complete). Returns the exit status, 0."""
            with report_lock:
                if rank == 0 and not report_early.done:
                    out = json.loads(json.dumps(result))
                    out["partitions"][name] = {"error": why, "note": notes[name.rstrip("0123456789")]}
                    print(json.dumps(out), flush=True)
                    report_early.done = True
            return 0
        report_early.done = False

        def leg_expired(name):
            # runs on the watchdog thread of a rank whose leg budget ran out (every rank's budget
            # starts at the same collective, so they expire together)
            return lambda phase: report_early(name, f"did not finish within {args.leg_seconds:.0f} s (phase '{phase}')")

        for part, groups in extra:
            name = part if groups is None else f"{part}{groups}"
            watchdog.leg(f"{name} leg", args.leg_seconds, leg_expired(name))
            leg, err = {"note": notes[part]}, None
            xshard = None
            try:
                if part != "params" and ensure_transport() is None:
                    raise TransportError(tstate["error"])
                watchdog.enter(f"{name} leg")
                saved, args.device_groups = args.device_groups, groups
                try:
                    if part == "weak":
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
                if xinfo.get("route"):
                    leg["halo_critical_MB"] = round(xinfo["route"]["critical_elems"] * 4 / 1e6, 1)
                    leg["halo_carved"] = xinfo.get("halo_carved")
                if xtune:
                    leg["autotune"] = xtune
                if part != "params":
                    leg["transport"] = tstate["transport"].name
                    leg["comparable"] = tstate["comparable"]
            except Exception as exc:  # reported in the line; every rank takes the same decision below
                err = f"{type(exc).__name__}: {exc}"
                print(f"[bench rank {rank}] {name} leg failed: {err}", file=sys.stderr, flush=True)
            finally:
                xshard = None
                drop_cached()
            try:
                all_ok = agree_all(err is None)
            except Exception as exc:  # a peer has left (its leg budget ran out first): report and end
                print(f"[bench rank {rank}] control plane lost a peer in the {name} leg ({exc})",
                      file=sys.stderr, flush=True)
                os._exit(report_early(name, err or f"a rank left during the leg ({type(exc).__name__})"))
            if not all_ok:
                leg = {"error": err or "failed on another rank", "note": notes[part]}
            legs[name] = leg
            watchdog.end_leg()
        if rank == 0 and not legs:
            result.pop("partitions", None)
    if world > 1:
        dist.barrier()
    # CPU baselines: rank 0, N = 1 only (bounded samples).
    watchdog.enter("baselines and report")
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(P, K, args.cpu_seconds)
            if args.cpu_pool_seconds > 0:
                result["cpu_baseline_pool"] = cpu_baseline_pool(P, K, D, args.cpu_pool_seconds)
        else:
            result["cpu_baseline"] = None
        if not args.no_live_traffic and not args.window_batch:
            # N > 1: the rank's own shape (its devices, its element slice) as a whole ring round,
            # since short rows are partly re-read from the Infinity Cache (rows_note)
            live, note = live_traffic(shard_P(info, P), K, ring=info["devices_per_rank"] if world > 1 else 0)
            rl = result["roofline"]
            if live is not None:
                rl["traffic_committed"] = rl["traffic"]
                rl["traffic"] = round(live, 1)
                rl["traffic_over_algorithmic"] = round(live / rl["bytes_per_launch"], 5)
            rl["traffic_source"] = note if live is not None else f"committed profile ({note})"
        if args.e2e and world == 1:
            from federated_amd.staging import measure_e2e
            result["e2e"] = measure_e2e(eng, P, K)
        print(json.dumps(result), flush=True)
    if tstate["transport"] is not None:
        tstate["transport"].close()
    if world > 1:
        dist.destroy_process_group()
    watchdog.done()


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


def shard_P(info, P):
    lo, hi = info["slice"]
    return hi - lo


if __name__ == "__main__":
    main()
