"""The sharded BASELINE configs through the HIP path: every shard's kernels on one MI355X, the
cross-shard halo over the in-process loopback transport (federated_amd/loopback.py: one host
thread per shard, device-to-device hipMemcpyAsync with the per-pair issue-order pairing of
cfa_p2p_group_f32), several rounds with the mixed models fed back, every device checked bit for
bit against the unsharded oracle trajectory.

- C4: CIFAR-100 VGG-1 buckets (P = 1 071 748), 32 devices, K = 4, 4 shards
  (TF2 CIFAR100_dataset/...FL_threads_CIFAR100.py:160-170,442-450; consensus_v3.py:44-70 window
  and the drivers' np.random.choice lists).
- C5: radar buckets (P = 24 622), 128 devices on the v4 ring (N < 2: in-neighbour ii - 1,
  consensus_v4.py:133-137), 8 shards, the bench's routed (relayed, staged) exchange.
- The bench's own N = 8 plan (128 devices, K = 8 ring window, relayed + staged halo) at a
  reduced bucket size, and the sharded FedAvg all-reduce (parameter_server_v2.py:159-161).
RCCL itself never runs at world > 1 on a one-GPU box; the loopback stands in for it here.
"""
import numpy as np
import pytest
import torch

from oracle.cfa_oracle import ps_fedavg, sequential_mix, tf2_kregular_v3, tf2_kregular_v4

pytestmark = pytest.mark.gpu


def _seed_full(D, P, base):
    return [torch.randn(P, generator=torch.Generator().manual_seed(base + g)).numpy() for g in range(D)]


def _oracle_trajectory(full, lists, alphas_of, rounds):
    cur = [x.copy() for x in full]
    for _ in range(rounds):
        cur = [sequential_mix(cur[d], [cur[j] for j in lists[d]], alphas_of(d)) for d in range(len(cur))]
    return cur


def _c4_lists(topology, D, K):
    if topology == "kregular_v3":
        return [tf2_kregular_v3(d, K, D).tolist() for d in range(D)]
    rng = np.random.default_rng(2026)
    return [[int(j) for j in rng.choice([k for k in range(D) if k != d], K, replace=False)] for d in range(D)]


@pytest.mark.parametrize("topology", ["kregular_v3", "random_choice"])
def test_c4_sharded_4_ranks_loopback(gpu, topology):
    from federated_amd.graph_population import GraphPopulationShard, GraphShardPlan
    from loopback import LoopbackHub, run_ranks
    D, K, world, P, rounds = 32, 4, 4, 1_071_748, 3
    lists = _c4_lists(topology, D, K)
    full = _seed_full(D, P, 4400)

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
        return plan.first, shard.models.cpu().numpy(), len(plan.halo_devices)

    hub = LoopbackHub(world)
    res = run_ranks(world, rank_fn, hub=hub)
    assert sum(hub.messages) > 0 and all(h > 0 for _, _, h in res)  # the halo really moved
    ref = _oracle_trajectory(full, lists, lambda d: [1.0 / (len(lists[d]) + 1)] * len(lists[d]), rounds)
    for first, block, _ in res:
        for i in range(block.shape[0]):
            assert np.array_equal(block[i], ref[first + i]), (topology, first + i)


def _ring_sharded(gpu, world, D, hl, hr, P, rounds, base, relay=True, staged=True, partition="devices",
                  dev_groups=None, slices=False):
    from loopback import LoopbackHub, run_ranks
    from federated_amd.population import make_ring_shard
    full = _seed_full(D, P, base)

    def rank_fn(rank, transport):
        shard, info = make_ring_shard(rank, world, D, hl, hr, P, torch.device("cuda"), transport, gpu,
                                      partition=partition, dev_groups=dev_groups, relay=relay, staged=staged)
        lo, hi = info["slice"]
        cs, ms = torch.cuda.Stream(), torch.cuda.Stream()
        with torch.cuda.stream(cs):
            for i in range(shard.plan.L):
                shard.models[i].copy_(torch.from_numpy(full[shard.plan.first + i][lo:hi]))
            for _ in range(rounds):
                shard.round(cs, ms)
                shard.models.copy_(shard.mixed)
        cs.synchronize()
        if slices:
            return shard.plan.first, shard.models.cpu().numpy(), info.get("route"), shard.alphas, (lo, hi)
        return shard.plan.first, shard.models.cpu().numpy(), info.get("route"), shard.alphas

    hub = LoopbackHub(world)
    res = run_ranks(world, rank_fn, hub=hub)
    return full, res, hub


def test_c5_radar_ring_sharded_8_ranks_loopback(gpu):
    D, world, P, rounds = 128, 8, 24_622, 3
    full, res, hub = _ring_sharded(gpu, world, D, 1, 0, P, rounds, 5500)
    assert res[0][2]["relay"] in (True, False) and sum(hub.messages) >= world * rounds
    lists = [[int(tf2_kregular_v4(d, 1, D))] for d in range(D)]
    assert all(r[3] == [0.5] for r in res)  # consensus_v4 eps for one neighbour
    ref = _oracle_trajectory(full, lists, lambda d: [0.5], rounds)
    for first, block, _, _ in res:
        for i in range(block.shape[0]):
            assert np.array_equal(block[i], ref[first + i]), first + i


def test_bench_plan_n8_loopback_reduced_bucket(gpu):
    """bench.py's N = 8 schedule (128 devices, K = 8 ring window, relayed + staged routed halo)
    with every shard's streaming mixes on this GPU, at P = 1M instead of 25M."""
    D, world, P, rounds, h = 128, 8, 1_000_003, 2, 4
    full, res, hub = _ring_sharded(gpu, world, D, h, h, P, rounds, 6600)
    assert res[0][2]["relay"] is True
    lists = [[(d + o) % D for o in list(range(-h, 0)) + list(range(1, h + 1))] for d in range(D)]
    ref = _oracle_trajectory(full, lists, lambda d: [1.0 / (2 * h + 1)] * (2 * h), rounds)
    for first, block, _, _ in res:
        for i in range(block.shape[0]):
            assert np.array_equal(block[i], ref[first + i]), first + i


@pytest.mark.parametrize("world,partition,groups", [(4, "hybrid", 2), (8, "hybrid", 4), (4, "params", None)])
def test_ring_partitions_loopback(gpu, world, partition, groups):
    """The bench's other partitions (element slices; device blocks x element slices with the
    routed halo between ranks holding the same slice), every shard's mixes on this GPU, two rounds
    fed back, each rank's slice of its devices bit-exact with the unsharded oracle."""
    D, P, rounds, h = 32, 262_147, 2, 4
    full, res, hub = _ring_sharded(gpu, world, D, h, h, P, rounds, 8800, partition=partition, dev_groups=groups,
                                   slices=True)
    lists = [[(d + o) % D for o in list(range(-h, 0)) + list(range(1, h + 1))] for d in range(D)]
    ref = _oracle_trajectory(full, lists, lambda d: [1.0 / (2 * h + 1)] * (2 * h), rounds)
    covered = np.zeros((D, P), dtype=bool)
    for first, block, _, _, (lo, hi) in res:
        for i in range(block.shape[0]):
            assert np.array_equal(block[i], ref[first + i][lo:hi]), (partition, first + i, lo)
            covered[first + i, lo:hi] = True
    assert covered.all()  # the ranks' blocks and slices tile the whole population
    if partition == "hybrid":
        assert sum(hub.messages) > 0


def test_sharded_fedavg_4_ranks_loopback(gpu):
    """ShardedFedAvg over 4 shards: libcfa's linear pre-scaling launch on every shard, the
    loopback sum all-reduce; within the documented 1e-5 normwise of the sequential fold."""
    from loopback import run_ranks
    from federated_amd.ps_shard import ShardedFedAvg
    world, D, P = 4, 10, 262_147
    models = _seed_full(D, P, 7700)
    params = _seed_full(1, P, 7799)[0]

    def rank_fn(rank, t):
        fa = ShardedFedAvg(rank, world, D, P, "cuda", t, gpu, update_factor=0.9)
        fa.params.copy_(torch.from_numpy(params))
        for g in range(fa.first, fa.last):
            fa.models[g - fa.first].copy_(torch.from_numpy(models[g]))
        out = fa.aggregate(stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        return out.cpu().numpy()

    out = run_ranks(world, rank_fn)
    ref = np.asarray(ps_fedavg([params], [[m] for m in models], 0.9)[0])
    for b in out:
        assert np.array_equal(b, out[0])
        assert np.abs(b.astype(np.float64) - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.parametrize("partition,groups", [("devices", None), ("hybrid", 2)])
def test_bench_plan_n8_loopback_full_bucket(gpu, partition, groups):
    """bench.py's N = 8 plans at the BASELINE bucket size (128 devices x 25M fp32, K = 8 ring
    window): the relayed, staged device-block plan and the hybrid (2 device blocks x 4 element
    slices). One sharded round over the loopback equals the unsharded population round on the same
    GPU row for row (halo rows, relay slots and slices at their full-size offsets), and two
    boundary devices of the unsharded round equal the CPU oracle."""
    from loopback import LoopbackHub, run_ranks
    from federated_amd.population import make_ring_shard
    D, world, P, h, base = 128, 8, 25_000_000, 4, 9900
    dev = torch.device("cuda")

    def seed(t, g, lo, hi):
        gen = torch.Generator(device=dev).manual_seed(base + g)
        if (lo, hi) == (0, P):
            t.normal_(generator=gen)
            return
        full = torch.empty(P, dtype=torch.float32, device=dev)
        full.normal_(generator=gen)
        t.copy_(full[lo:hi])

    ref, _ = make_ring_shard(0, 1, D, h, h, P, dev, None, gpu)
    for g in range(D):
        seed(ref.models[g], g, 0, P)
    ref.round()
    torch.cuda.synchronize()

    def rank_fn(rank, transport):
        shard, info = make_ring_shard(rank, world, D, h, h, P, dev, transport, gpu, partition=partition,
                                      dev_groups=groups)
        lo, hi = info["slice"]
        cs, ms = torch.cuda.Stream(), torch.cuda.Stream()
        with torch.cuda.stream(cs):
            for i in range(shard.plan.L):
                seed(shard.models[i], shard.plan.first + i, lo, hi)
            shard.round(cs, ms)
        cs.synchronize()
        bad = [shard.plan.first + i for i in range(shard.plan.L)
               if not torch.equal(shard.mixed[i], ref.mixed[shard.plan.first + i][lo:hi])]
        return bad, info.get("route"), (lo, hi), shard.plan.first, shard.plan.L

    hub = LoopbackHub(world)
    res = run_ranks(world, rank_fn, hub=hub)
    assert sum(hub.messages) > 0
    assert all(not bad for bad, *_ in res), [bad for bad, *_ in res]
    covered = np.zeros(D, dtype=np.int64)
    for _, _, (lo, hi), first, L in res:
        covered[first:first + L] += hi - lo
    assert (covered == P).all()  # blocks and slices tile every bucket exactly once
    if partition == "devices":
        assert res[0][1]["relay"] is True
    alphas = [1.0 / (2 * h + 1)] * (2 * h)
    for g in (15, 16):  # the last device of rank 0's block and the first of rank 1's
        rows = [ref.models[(g + o) % D].cpu().numpy() for o in list(range(-h, 0)) + list(range(1, h + 1))]
        want = sequential_mix(ref.models[g].cpu().numpy(), rows, alphas)
        assert np.array_equal(ref.mixed[g].cpu().numpy(), want), g
        del rows, want
    del ref
    torch.cuda.empty_cache()
