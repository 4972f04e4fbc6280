"""CPU tests of the in-process loopback transport (federated_amd/loopback.py): the sharded
population's exchange schedules run through it with host buffers, one thread per rank.

The same schedules run on the GPU, every shard's HIP kernels on one card, in
tests/test_gpu_sharded_configs.py (C4 over 4 shards, C5 over 8)."""
import numpy as np
import pytest
import torch

from federated_amd.graph_population import GraphPopulationShard, GraphShardPlan
from loopback import LoopbackError, LoopbackHub, run_ranks
from federated_amd.population import make_ring_shard
from oracle.cfa_oracle import sequential_mix, tf2_kregular_v3


def _seeded(g, P):
    return torch.randn(P, generator=torch.Generator().manual_seed(9100 + g))


@pytest.mark.parametrize("world,D,h,hr,partition,gd,relay,staged", [
    (8, 64, 4, 4, "devices", None, True, True),     # the bench's relayed, staged plan at world 8
    (8, 64, 4, 4, "devices", None, True, False),
    (4, 16, 4, 4, "devices", None, False, True),
    (8, 32, 4, 4, "hybrid", 4, True, True),
    (8, 128, 1, 0, "devices", None, True, True),    # C5: v4 ring (in-neighbour ii-1) over 8 ranks
    (2, 16, 4, 4, "devices", None, True, True),     # world 2: left and right peer coincide
])
def test_routed_ring_exchange_loopback(world, D, h, hr, partition, gd, relay, staged):
    """Every rank's halo after the routed exchange equals the unsharded population's buckets, and
    every boundary mix equals the oracle's."""
    P = 515
    full = [_seeded(g, P) for g in range(D)]

    def rank_fn(rank, transport):
        shard, info = make_ring_shard(rank, world, D, h, hr, P, "cpu", transport, None, partition=partition,
                                      dev_groups=gd, relay=relay, staged=staged)
        lo, hi = info["slice"]
        for i in range(shard.plan.L):
            shard.models[i] = full[shard.plan.first + i][lo:hi]
        shard.exchange()
        ok = True
        for i in range(shard.plan.L):
            g = shard.plan.first + i
            nb = shard.plan.neighbours(g)
            srcs = [s.numpy() for s in shard.sources(i)]
            ok &= all(np.array_equal(s, full[j][lo:hi].numpy()) for s, j in zip(srcs, nb))
            ref = sequential_mix(full[g].numpy(), [full[j].numpy() for j in nb], shard.alphas)[lo:hi]
            ok &= np.array_equal(sequential_mix(shard.models[i].numpy(), srcs, shard.alphas), ref)
        route = shard._route_plan
        return ok, (len(route.groups) if route is not None else 0), info.get("route_digest")

    hub = LoopbackHub(world, timeout=60)
    res = run_ranks(world, rank_fn, hub=hub)
    assert all(ok for ok, _, _ in res)
    assert len({d for _, _, d in res}) == 1
    # one exchange call per route group on every rank (the RCCL group count of the same plan)
    groups = [g for _, g, _ in res]
    assert hub.groups == groups if partition != "params" else True


@pytest.mark.parametrize("topology", ["kregular_v3", "random_choice"])
def test_graph_population_exchange_loopback_c4_shape(topology):
    """C4's topology (32 devices, K = 4) over 4 ranks: the grouped halo of GraphPopulationShard
    through the loopback; every halo row equals the owner's bucket."""
    D, K, world, P = 32, 4, 4, 257
    if topology == "kregular_v3":
        lists = [tf2_kregular_v3(d, K, D).tolist() for d in range(D)]
    else:
        rng = np.random.default_rng(2026)
        lists = [[int(j) for j in rng.choice([k for k in range(D) if k != d], K, replace=False)] for d in range(D)]
    full = [_seeded(g, P) for g in range(D)]

    def rank_fn(rank, transport):
        plan = GraphShardPlan(lists, rank, world)
        shard = GraphPopulationShard(plan, P, "cpu", transport, None)
        for i in range(plan.L):
            shard.models[i] = full[plan.first + i]
        shard.exchange()
        return all(torch.equal(shard.halo[h], full[g]) for h, g in enumerate(plan.halo_devices))

    assert all(run_ranks(world, rank_fn))


def test_fifo_pairing_and_zero_length_messages():
    """Messages between one pair pair up in issue order; zero-length ones are skipped on both
    sides; a self message works."""
    def rank_fn(rank, t):
        if rank == 0:
            a, b, z = torch.arange(5.0), torch.arange(3.0) + 10, torch.empty(0)
            me_out, me_in = torch.tensor([7.0, 8.0]), torch.empty(2)
            t.exchange([(a, 1), (z, 1), (b, 1), (me_out, 0)], [(me_in, 0)])
            return me_in.tolist()
        x, y, z = torch.empty(5), torch.empty(3), torch.empty(0)
        t.exchange([], [(z, 0), (x, 0), (y, 0)])
        return x.tolist(), y.tolist()

    r0, r1 = run_ranks(2, rank_fn)
    assert r0 == [7.0, 8.0]
    assert r1 == ([0.0, 1.0, 2.0, 3.0, 4.0], [10.0, 11.0, 12.0])


def test_mismatched_lengths_fail_both_sides():
    def rank_fn(rank, t):
        if rank == 0:
            t.exchange([(torch.zeros(4), 1)], [])
        else:
            t.exchange([], [(torch.empty(5), 0)])

    with pytest.raises(LoopbackError, match="sent 4 floats"):
        run_ranks(2, rank_fn, hub=LoopbackHub(2, timeout=20))


def test_missing_peer_times_out_with_the_pair_named():
    def rank_fn(rank, t):
        if rank == 1:
            t.exchange([], [(torch.empty(3), 0)])

    with pytest.raises(LoopbackError, match="from rank 0 to rank 1"):
        run_ranks(2, rank_fn, hub=LoopbackHub(2, timeout=1))


def test_failure_ends_peer_waits_early():
    """A rank that fails ends the other ranks' waits with its message (no full timeout)."""
    import time

    def rank_fn(rank, t):
        if rank == 0:
            raise RuntimeError("boom")
        t.exchange([], [(torch.empty(3), 0)])

    t0 = time.perf_counter()
    with pytest.raises(RuntimeError, match="boom"):
        run_ranks(3, rank_fn, hub=LoopbackHub(3, timeout=60))
    assert time.perf_counter() - t0 < 10


@pytest.mark.parametrize("root", [None, 2])
def test_allreduce_and_reduce_sum_rank_order(root):
    world = 4
    vals = [torch.randn(33, generator=torch.Generator().manual_seed(r)) for r in range(world)]
    ref = vals[0].clone()
    for v in vals[1:]:
        ref += v

    def rank_fn(rank, t):
        buf = vals[rank].clone()
        for _ in range(3):  # generations do not mix
            b = buf.clone()
            if root is None:
                t.allreduce_sum(b)
            else:
                t.reduce_sum(b, root)
        return b

    out = run_ranks(world, rank_fn)
    for r, b in enumerate(out):
        if root is None or r == root:
            assert torch.equal(b, ref)
        else:
            assert torch.equal(b, vals[r])


def test_sharded_fedavg_loopback_cpu():
    """ShardedFedAvg over 4 in-process ranks (the loopback all-reduce) within the documented
    1e-5 normwise of the reference's sequential fold (oracle.ps_fedavg)."""
    from federated_amd.ps_shard import ShardedFedAvg
    from oracle.cfa_oracle import ps_fedavg

    class NumpyEngine:  # host stand-in for the linear mix (the GPU test uses libcfa)
        def mix_linear(self, out, local, nbrs, coeff, stream=None):
            acc = local.double() * coeff[0]
            for c, x in zip(coeff[1:], nbrs):
                acc += x.double() * c
            out.copy_(acc.float())

    world, D, P = 4, 10, 301
    models = [_seeded(g, P) for g in range(D)]
    params = _seeded(99, P)

    def rank_fn(rank, t):
        fa = ShardedFedAvg(rank, world, D, P, "cpu", t, NumpyEngine(), update_factor=0.9)
        fa.params.copy_(params)
        for g in range(fa.first, fa.last):
            fa.models[g - fa.first] = models[g]
        return fa.aggregate().clone()

    out = run_ranks(world, rank_fn)
    ref = np.asarray(ps_fedavg([params.numpy()], [[m.numpy()] for m in models], 0.9)[0])
    for b in out:
        assert torch.equal(b, out[0])
        d = np.abs(b.numpy().astype(np.float64) - ref).max()
        assert d <= 1e-5 * np.abs(ref).max()


def test_the_first_failure_is_the_one_raised():
    """Rank 2 fails; ranks 0 and 1 then give up waiting. run_ranks raises rank 2's error."""
    def rank_fn(rank, t):
        if rank == 2:
            raise ValueError("the cause")
        t.exchange([], [(torch.empty(3), 2)])

    with pytest.raises(ValueError, match="the cause"):
        run_ranks(3, rank_fn, hub=LoopbackHub(3, timeout=30))
