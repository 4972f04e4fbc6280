"""Randomised sharded populations through the HIP path on one GPU: every shard's kernels on this
MI355X, the cross-shard halo over the in-process loopback transport (tests/loopback.py, the
per-pair issue-order pairing of cfa_p2p_group_f32), two rounds with the mixed models fed back,
every device (and every element slice) checked bit for bit against the unsharded oracle
trajectory. The fixed configs are in test_gpu_sharded_configs.py; here the world size, the
population, the window, the partition, the routing and the bucket size are drawn at random:

- ring populations (population.make_ring_shard, bench.py's shard): world 2..8, D a multiple of
  the device groups, h_left / h_right 0..4, partitions devices / params / hybrid, relayed or
  direct halo, staged or not, P from 64 to 300K (odd sizes included);
- any-topology populations (graph_population.GraphPopulationShard): world 2..6, random lists
  (the CSR halo plan), blocks of unequal size.

References: the ring window of cfa.py:14-32 / consensus_v4.py:133-137, the TF2 rule
consensus_v3.py:145,153-155. CFA_SHARD_FUZZ_CASES (default 12) sets the number of cases.
"""
import os

import numpy as np
import pytest
import torch

from test_gpu_sharded_configs import _oracle_trajectory, _ring_sharded, _seed_full

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("CFA_SHARD_FUZZ_CASES", "12"))
SEED0 = int(os.environ.get("CFA_SHARD_FUZZ_SEED", "73000"))


def _ring_case(rng):
    world = int(rng.integers(2, 9))
    partition = ["devices", "params", "hybrid"][int(rng.integers(0, 3))]
    groups = None
    if partition == "hybrid":
        divs = [g for g in range(2, world) if world % g == 0]
        if not divs:
            partition = "devices"
        else:
            groups = int(rng.choice(divs))
    gd = {"devices": world, "params": 1, "hybrid": groups}[partition]
    hl, hr = int(rng.integers(0, 5)), int(rng.integers(0, 5))
    L = max(1, hl, hr, int(rng.integers(1, 7)))
    D = gd * L
    while hl + hr >= D:
        D += gd
    P = int(rng.integers(64, 300_000))
    return world, partition, groups, D, hl, hr, P, bool(rng.random() < 0.7), bool(rng.random() < 0.7)


@pytest.mark.parametrize("case", range(CASES))
def test_ring_shards_fuzz(gpu, case):
    rng = np.random.default_rng(SEED0 + case)
    world, partition, groups, D, hl, hr, P, relay, staged = _ring_case(rng)
    info = (world, partition, groups, D, hl, hr, P, relay, staged)
    rounds = 2
    full, res, hub = _ring_sharded(gpu, world, D, hl, hr, P, rounds, 12000 + case, relay=relay, staged=staged,
                                   partition=partition, dev_groups=groups, slices=True)
    lists = [[(d + o) % D for o in list(range(-hl, 0)) + list(range(1, hr + 1))] for d in range(D)]
    K = hl + hr
    ref = _oracle_trajectory(full, lists, lambda d: [1.0 / (K + 1)] * K, rounds)
    covered = np.zeros((D, P), dtype=bool)
    for first, block, _, _, (lo, hi) in res:
        for i in range(block.shape[0]):
            assert np.array_equal(block[i], ref[first + i][lo:hi]), info + (first + i, lo)
            covered[first + i, lo:hi] = True
    assert covered.all(), info


@pytest.mark.parametrize("case", range(max(1, CASES // 2)))
def test_graph_shards_fuzz(gpu, case):
    from federated_amd.graph_population import GraphPopulationShard, GraphShardPlan
    from loopback import LoopbackHub, run_ranks
    rng = np.random.default_rng(SEED0 + 500 + case)
    world = int(rng.integers(2, 7))
    D = int(rng.integers(world, 5 * world + 1))
    lists = [[int(j) for j in rng.choice([k for k in range(D) if k != d], int(rng.integers(0, min(6, D - 1) + 1)),
                                         replace=False)] for d in range(D)]
    P = int(rng.integers(64, 200_000))
    rounds = 2
    full = _seed_full(D, P, 15000 + case)

    def rank_fn(rank, transport):
        plan = GraphShardPlan(lists, rank, world)
        shard = GraphPopulationShard(plan, P, "cuda", transport, gpu)
        cs, ms = torch.cuda.Stream(), torch.cuda.Stream()
        with torch.cuda.stream(cs):
            for i in range(plan.L):
                shard.models[i].copy_(torch.from_numpy(full[plan.first + i]))
            for _ in range(rounds):
                shard.round(cs, ms)
                shard.models.copy_(shard.mixed)
        cs.synchronize()
        return plan.first, shard.models.cpu().numpy()

    res = run_ranks(world, rank_fn, hub=LoopbackHub(world))
    ref = _oracle_trajectory(full, lists, lambda d: [1.0 / (len(lists[d]) + 1)] * len(lists[d]), rounds)
    seen = 0
    for first, block in res:
        for i in range(block.shape[0]):
            assert np.array_equal(block[i], ref[first + i]), (world, D, P, first + i)
            seen += 1
    assert seen == D
