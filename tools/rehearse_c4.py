#!/usr/bin/env python3
"""Config 4 (CIFAR-100 VGG-1 buckets, P = 1 071 748, 32 devices, K = 4) as a sharded population
trajectory: GraphPopulationShard over N ranks (launched by torch.distributed.run; on a one-GPU
box every rank shares the card and the halo goes over gloo, host-staged), R rounds with the
mixed models fed back, every rank's block checked bit for bit against the unsharded population
run on the same GPU. Two topologies: the TF2 k-regular window and seeded random neighbour lists
(the drivers' np.random.choice rule), whose halos reach non-adjacent ranks.

Usage: python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \\
           --master-port 29650 tools/rehearse_c4.py [--rounds 3]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from federated_amd import topology as T  # noqa: E402
from federated_amd.dist import TorchTransport  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.graph_population import GraphPopulationShard, GraphShardPlan  # noqa: E402


def seeded(shard, P):
    gen = torch.Generator(device="cuda")
    for i in range(shard.plan.L):
        gen.manual_seed(4000 + shard.plan.first + i)
        shard.models[i].normal_(generator=gen)


def trajectory(shard, rounds, comm=None):
    for _ in range(rounds):
        shard.round(torch.cuda.current_stream(), comm)
        shard.models.copy_(shard.mixed)
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--params", type=int, default=1_071_748)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    eng = get_engine(0)
    D, K, P = 32, 4, a.params
    rng = np.random.default_rng(2026)
    topologies = {
        "kregular_v3": T.kregular_v3(D, K),
        "random_choice": [[int(j) for j in rng.choice([k for k in range(D) if k != d], K, replace=False)]
                          for d in range(D)],
    }
    report = {}
    for name, lists in topologies.items():
        plan = GraphShardPlan(lists, rank, world)
        shard = GraphPopulationShard(plan, P, "cuda", TorchTransport(), eng)
        seeded(shard, P)
        trajectory(shard, a.rounds, torch.cuda.Stream())
        ref = GraphPopulationShard(GraphShardPlan(lists, 0, 1), P, "cuda", None, eng)
        seeded(ref, P)
        trajectory(ref, a.rounds)
        ok = torch.equal(shard.models, ref.models[plan.first:plan.first + plan.L])
        flag = torch.tensor([int(ok)], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        report[name] = {"halo_devices_rank0": len(plan.halo_devices) if rank == 0 else None,
                        "all_ranks_bit_exact": bool(flag.item())}
        del shard, ref
        torch.cuda.empty_cache()
    if rank == 0:
        print(json.dumps({"experiment": "tools/rehearse_c4.py", "ranks": world, "devices": D, "K": K, "P": P,
                          "rounds": a.rounds, "transport": "torch (gloo), all ranks on one GPU",
                          "topologies": report}), flush=True)
    dist.destroy_process_group()
    if not all(r["all_ranks_bit_exact"] for r in report.values()):
        sys.exit(1)


if __name__ == "__main__":
    main()
