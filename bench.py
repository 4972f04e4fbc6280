#!/usr/bin/env python3
"""Benchmark: device-resident CFA reduction of K neighbour fp32 buckets on MI355X.

Metric (BASELINE.json): "device-resident GB/s, CFA reduce of K neighbour fp32 param buckets;
1/2/4/8 GPU". Workload (BASELINE.json north_star target): 8 neighbour buckets x 25M fp32 params
mixed into each device's local model (the TF2 sequential CFA rule, eps = 1/(K+1),
consensus_v3.py:145,153-155). The simulated device population is sharded one shard per GPU
(weak scaling): each rank owns ``--devices-per-gpu`` devices on a wrap-around ring window of
K = 8 neighbours; one step = one consensus round of the shard = RCCL halo exchange of the 2x4
boundary buckets (N > 1) overlapped with the interior mixes, then the boundary mixes.

value = algorithmic bytes of all mixes on all ranks / max-over-ranks wall time, with
algorithmic bytes = (K + 2) * P * 4 per device mix (K neighbour reads + local read + output
write). Inputs are resident in HBM when the timed region starts.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU; RANK/LOCAL_RANK/WORLD_SIZE from the environment).
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
    p.add_argument("--devices-per-gpu", type=int, default=128,
                   help="simulated devices per GPU (128 x 100 MB models + outputs = 26 GB of HBM)")
    p.add_argument("--transport", default="rccl", choices=["rccl", "torch"])
    p.add_argument("--window-batch", type=int, default=0,
                   help="B > 0: mix B consecutive devices per cfa_mix_window_f32 pass (each window row "
                        "loaded once); 0 (default) = one streaming mix per device, the judged kernel")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--traffic-json", default=None,
                   help="PMC traffic summary (default profiles/r01_pmc_traffic.json, or "
                        "profiles/r01_window_pmc_traffic.json with --window-batch)")
    p.add_argument("--e2e", action="store_true",
                   help="also measure the host-resident path (pinned H2D + mix + D2H) on rank 0")
    return p.parse_args()


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


def open_transport(kind, rank, world, device):
    """The requested transport; if it cannot be opened, torch.distributed P2P over an nccl
    (= RCCL) group, then over the gloo group (host-staged) as the last resort. The transport
    used is reported in the JSON config."""
    import torch.distributed as dist
    from federated_amd.dist import TorchTransport, make_transport
    import torch

    def agree(ok: int) -> bool:  # every rank takes the same decision (MIN over the gloo group)
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return int(flag.item()) == 1

    t, ok = None, 1
    try:
        t = make_transport(kind, rank, world, device)
    except Exception as exc:
        ok = 0
        print(f"[bench rank {rank}] {kind} transport failed ({exc})", file=sys.stderr)
    if agree(ok):
        return t
    if t is not None:
        t.close()
    # torch P2P over an nccl (= RCCL) group: its communicator is created lazily, so probe it with
    # one all-reduce before trusting it
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
        return t
    t = TorchTransport()
    t.name = "torch-gloo"
    return t


def main():
    args = parse()
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
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from federated_amd.engine import get_engine
    from federated_amd.population import RingPopulationShard, RingShardPlan

    P, K, L = args.params, args.neighbours, args.devices_per_gpu
    if K % 2:
        sys.exit("--neighbours must be even (ring window K/2 per side)")
    eng = get_engine(device)
    plan = RingShardPlan(rank, world, L, K // 2)
    transport = None
    if world > 1:
        transport = open_transport(args.transport, rank, world, device)
    shard = RingPopulationShard(plan, P, torch.device("cuda", device), transport, eng,
                                window_batch=args.window_batch)

    gen = torch.Generator(device=shard.device)
    for i in range(L):  # synthetic models: seeded per global device id
        gen.manual_seed(20261015 + plan.first + i)
        shard.models[i].normal_(generator=gen)

    compute = torch.cuda.current_stream()
    comm = torch.cuda.Stream() if world > 1 else None

    # Dominant-kernel timing, live in the timed region: one HIP event pair per step around the
    # back-to-back interior mixes on the stream they run on (no events between launches, so
    # the measurement does not perturb the round); avg launch = batch time / launches. This
    # includes the sub-microsecond kernel boundaries, so it is a conservative (upper) bound on
    # the kernel duration that rocprofv3 reports.
    interior = plan.interior()
    first_i, last_i = interior[0], interior[-1]
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    step_idx = [0]

    def timer(i, start):
        if start and i == first_i:
            ev[step_idx[0]][0].record(compute)
        elif not start and i == last_i:
            ev[step_idx[0]][1].record(compute)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        shard.round(compute, comm)
    barrier()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step_idx[0] = s
        shard.round(compute, comm, timer)
    barrier()
    elapsed = time.perf_counter() - t0
    launches_per_step = len(shard.window_passes(interior)) if args.window_batch else len(interior)
    durations = [a.elapsed_time(b) / launches_per_step for a, b in ev]
    launches_timed = launches_per_step * args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    bytes_total = world * shard.bytes_per_round * args.steps
    value = bytes_total / elapsed / 1e9
    per_launch_bytes = (K + 2) * P * 4 * len(interior) // launches_per_step  # algorithmic, per launch
    avg_ms = sum(durations) / max(1, len(durations))
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0

    result = None
    if rank == 0:
        result = {
            "metric": "device-resident GB/s, CFA reduce of K neighbour fp32 param buckets; 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded torch normal fp32 buckets, resident in HBM)",
            "config": {
                "workload": ("cfa_population_round (window passes of %d devices, rows loaded once per pass): "
                             % args.window_batch if args.window_batch else "cfa_population_round: ") +
                            "sequential CFA mix (eps=1/(K+1)) of every device "
                            "with K ring-window neighbours, devices sharded one shard per GPU",
                "params_per_bucket": P,
                "neighbours": K,
                "devices_per_gpu": L,
                "devices_total": plan.D,
                "bytes_per_device_mix": (K + 2) * P * 4,
                "window_batch": args.window_batch,
                "transport": transport.name if transport else "none",
                "parallelism": f"population-shard{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "window_vec_kernel" if args.window_batch else KERNEL,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "avg_launch_ms": round(avg_ms, 5),
                "step_avg_launch_ms_median": round(statistics.median(durations), 5) if durations else None,
                "step_avg_launch_ms_min": round(min(durations), 5) if durations else None,
                "launches_timed": launches_timed,
                "timing": "HIP events around each step's back-to-back interior mixes / launches",
                "traffic": load_traffic(
                    args.traffic_json or os.path.join(ROOT, "profiles", "r01_window_pmc_traffic.json"
                                                      if args.window_batch else "r01_pmc_traffic.json"),
                    P, K, "window_vec_kernel" if args.window_batch else KERNEL,
                    args.window_batch or 1),
            },
        }
    if world > 1:
        dist.barrier()
    # CPU baseline: rank 0, N = 1 only (bounded sample).
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(P, K, args.cpu_seconds)
        else:
            result["cpu_baseline"] = None
        if args.e2e:
            from federated_amd.staging import measure_e2e
            result["e2e"] = measure_e2e(eng, P, K)
        print(json.dumps(result), flush=True)
    if transport is not None:
        transport.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
