"""CPU tests of the routed halo exchange (federated_amd/halo.py) and the strong-scaling
partitions of the ring population (population.make_ring_shard).

- Plan invariants for every world size 2..8 and both partitions with an exchange: per rank pair
  and group, the sender's messages and the receiver's pair up one to one in order and length
  (what RCCL needs to match them); every transfer's element range is delivered exactly once;
  relay slots of one stage never overlap; the schedule is deterministic.
- gloo runs at world 2, 4 and 8 (one process per rank, the N > 1 path's logic): after the
  routed exchange every halo row equals the neighbour bucket the unsharded population holds,
  and every device's mix equals the unsharded oracle's, for the devices, hybrid and params
  partitions, with and without relays.
"""
import os
from collections import defaultdict

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from federated_amd.halo import DIRECT, RoutePlan, ring_transfers, route_shares
from federated_amd.population import make_ring_shard, partition_shape, slice_bounds


def _check_plan(plan: RoutePlan):
    # pairing: per (group, src, dst) the send list on src equals the recv list on dst
    for g in range(len(plan.groups)):
        for a in range(plan.world):
            sends, _ = plan.rank_ops(a, g)
            for b in range(plan.world):
                _, recvs = plan.rank_ops(b, g)
                s = [m for m in sends if m.dst == b]
                r = [m for m in recvs if m.src == a]
                assert s == r
                assert all(m.count > 0 for m in s)
    # coverage: each transfer's [lo, hi) lands exactly once in its destination bucket
    landed = defaultdict(list)
    for msgs in plan.groups:
        for m in msgs:
            if not (isinstance(m.dst_key, tuple) and m.dst_key[0] == "relay"):
                landed[(m.dst, m.dst_key)].append((m.dst_off, m.dst_off + m.count))
    for t in plan.transfers:
        iv = sorted(landed.pop((t.dst, t.dst_key)))
        assert iv[0][0] == t.lo and iv[-1][1] == t.hi
        assert all(x[1] == y[0] for x, y in zip(iv, iv[1:]))
    assert not landed
    # relay slots: within a group, the first hops into one rank's slot do not overlap, and each
    # is read back by exactly one second hop in the next group with the same extent
    for g, msgs in enumerate(plan.groups):
        into = defaultdict(list)
        for m in msgs:
            if isinstance(m.dst_key, tuple) and m.dst_key[0] == "relay":
                assert m.dst_key == ("relay", g % 2)
                into[m.dst].append((m.dst_off, m.dst_off + m.count))
                assert m.dst_off + m.count <= plan.slot_elems(m.dst)
                nxt = [x for x in plan.groups[g + 1] if x.src == m.dst and x.src_key == m.dst_key
                       and x.src_off == m.dst_off]
                assert len(nxt) == 1 and nxt[0].count == m.count
        for ivs in into.values():
            ivs.sort()
            assert all(x[1] <= y[0] for x, y in zip(ivs, ivs[1:]))
    # every piece starts aligned
    for msgs in plan.groups:
        for m in msgs:
            assert m.src_off % plan.align == 0 and m.dst_off % plan.align == 0


@pytest.mark.parametrize("world", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("relay", [False, True])
def test_ring_route_plan_invariants(world, relay):
    D, P = 128 if 128 % world == 0 else 16 * world, 25_000
    tr = ring_transfers(world, D // world, 4, 4, P)
    plan = RoutePlan(world, tr, relay=relay)
    _check_plan(plan)
    assert plan.digest() == RoutePlan(world, tr, relay=relay).digest()
    if world < 3:
        assert not plan.relay
    # no link carries more than direct-only routing would put on it
    direct = RoutePlan(world, tr, relay=False)
    assert plan.critical_elems() <= direct.critical_elems()


@pytest.mark.parametrize("world,gd", [(4, 2), (8, 2), (8, 4)])
def test_hybrid_route_plan_invariants(world, gd):
    P = 10_007
    gp = world // gd
    b = slice_bounds(P, gp)
    tr = ring_transfers(gd, 32 // gd, 4, 4, P, slice_world=gp, slice_bounds=b)
    _check_plan(RoutePlan(world, tr, relay=True))


def test_relays_spread_the_halo_at_eight_ranks():
    """The cost model's input: at N = 8, D = 128, K = 8, P = 25M the busiest
    link of the routed exchange carries about half of what the direct exchange puts on each
    neighbour link, and the critical path (groups back to back) about 0.53x."""
    tr = ring_transfers(8, 16, 4, 4, 25_000_000)
    direct = RoutePlan(8, tr, relay=False)
    routed = RoutePlan(8, tr, relay=True)
    assert direct.max_link_elems() == 4 * 25_000_000
    assert routed.relay
    assert routed.max_link_elems() <= 0.55 * direct.max_link_elems()
    assert routed.critical_elems() <= 0.55 * direct.critical_elems()


def _uniform_rates(world, r=50.0):
    return {(a, b): r for a in range(world) for b in range(world) if a != b}


def test_equal_measured_costs_reproduce_the_uniform_plan():
    """Costs from equal rates scale every load alike: the same routes as no costs at all."""
    from federated_amd.halo import link_costs_from_rates
    tr = ring_transfers(8, 16, 4, 4, 25_000_000)
    costs = link_costs_from_rates(_uniform_rates(8))
    assert set(costs.values()) == {16}
    assert RoutePlan(8, tr, relay=True, link_cost=costs).digest() == RoutePlan(8, tr, relay=True).digest()


@pytest.mark.parametrize("slow", [(0, 1), (3, 2), (7, 0)])
def test_slow_link_sheds_pieces_and_keeps_pairing(slow):
    """Round-4 review item 2: with one directed link measured at a quarter of the others' rate,
    the measured-cost plan moves pieces off it (it carries less than on the uniform plan and less
    than the other neighbour links), the send/recv pairing and coverage invariants still hold, and
    its predicted exchange time at the measured rates beats the uniform plan's."""
    from federated_amd.halo import link_costs_from_rates
    world = 8
    tr = ring_transfers(world, 16, 4, 4, 25_000_000)
    rates = _uniform_rates(world)
    rates[slow] = 12.5
    costs = link_costs_from_rates(rates)
    assert costs[slow] == 64 and costs[(slow[1], slow[0])] == 16
    uniform = RoutePlan(world, tr, relay=True)
    measured = RoutePlan(world, tr, relay=True, link_cost=costs)
    _check_plan(measured)
    assert measured.link_elems[slow] < 0.5 * uniform.link_elems[slow]
    others = [measured.link_elems[(a, (a + 1) % world)] for a in range(world) if (a, (a + 1) % world) != slow]
    assert measured.link_elems[slow] < min(others)
    assert measured.predicted_ms(rates) < 0.8 * uniform.predicted_ms(rates)
    assert measured.critical_cost() <= RoutePlan(world, tr, relay=False, link_cost=costs).critical_cost()
    # the same costs give the same plan on every rank
    assert RoutePlan(world, tr, relay=True, link_cost=dict(costs)).digest() == measured.digest()


def test_direct_only_plan_with_a_slow_link_predicts_its_time():
    """Without relays the slow link's group sets the time: predicted_ms at the measured rates is
    the busiest group's bytes over the slow rate (the relay option is what removes it)."""
    world = 4
    tr = [t for t in ring_transfers(world, 8, 1, 1, 1_000_000)]
    tr = [type(t)(0, t.src, t.dst, t.src_key, t.dst_key, t.lo, t.hi) for t in tr]
    rates = _uniform_rates(world, 40.0)
    rates[(1, 2)] = 10.0
    plan = RoutePlan(world, tr, relay=False)
    assert plan.predicted_ms(rates) == pytest.approx(1_000_000 * 4 / 10e9 * 1e3)
    assert plan.predicted_ms(_uniform_rates(world, 40.0)) == pytest.approx(1_000_000 * 4 / 40e9 * 1e3)


def test_choose_route_keeps_the_fastest_predicted_plan():
    """halo.choose_route prices the uniform, rate-weighted and direct plans at the measured rates:
    equal or merely noisy rates (within the 15% tolerance) keep the uniform plan; one slow link
    picks the rate-weighted plan; every candidate's time is reported."""
    from federated_amd.halo import choose_route
    tr = ring_transfers(8, 16, 4, 4, 25_000_000)
    uniform = RoutePlan(8, tr, relay=True)
    plan, rep = choose_route(8, tr, relay=True, rates_gbps=_uniform_rates(8))
    assert rep["chosen"] == "uniform" and plan.digest() == uniform.digest()
    assert set(rep["candidates"]) == {"uniform", "direct"} and rep["slow_links"] == []
    noisy = {l: 50.0 * (0.9 + 0.02 * ((l[0] * 8 + l[1]) % 10)) for l in _uniform_rates(8)}
    plan, rep = choose_route(8, tr, relay=True, rates_gbps=noisy)
    assert rep["chosen"] == "uniform" and plan.digest() == uniform.digest()
    slow = _uniform_rates(8)
    slow[(2, 3)] = 10.0
    plan, rep = choose_route(8, tr, relay=True, rates_gbps=slow)
    assert rep["chosen"] == "measured" and rep["slow_links"] == ["2->3"]
    assert rep["candidates"]["measured"] < rep["candidates"]["uniform"] < rep["candidates"]["direct"]
    _check_plan(plan)
    plan, rep = choose_route(8, tr, relay=True, rates_gbps=None)
    assert rep["chosen"] == "uniform" and rep["candidates"] == {}


def test_choose_route_prices_the_per_message_cost():
    """With a large measured per-message cost, the plan with 16 parts per row (fewer messages)
    predicts a shorter exchange than 64 parts and is kept; with none, 16 parts are not even priced
    (they can only lengthen the byte critical path)."""
    from federated_amd.halo import choose_route
    tr = ring_transfers(8, 16, 4, 4, 25_000_000)
    rates = _uniform_rates(8)
    plan, rep = choose_route(8, tr, relay=True, rates_gbps=rates, message_us=0.0)
    assert set(rep["candidates"]) == {"uniform", "direct"} and plan.units == 64
    plan, rep = choose_route(8, tr, relay=True, rates_gbps=rates, message_us=200.0)
    assert set(rep["candidates"]) == {"uniform", "direct", "uniform/16", "direct/16"}
    assert rep["chosen"] in ("uniform/16", "direct", "direct/16") and rep["message_us"] == 200.0
    assert rep["candidates"][rep["chosen"]] == min(rep["candidates"].values())
    _check_plan(plan)
    m64 = RoutePlan(8, tr, relay=True)
    assert sum(m64.max_rank_messages(g) for g in range(len(m64.groups))) > \
        sum(plan.max_rank_messages(g) for g in range(len(plan.groups)))


def test_link_costs_reject_nonpositive_rates():
    from federated_amd.halo import link_costs_from_rates
    with pytest.raises(ValueError):
        link_costs_from_rates({(0, 1): 10.0, (1, 0): 0.0})
    assert link_costs_from_rates({}) == {}
    with pytest.raises(ValueError):
        RoutePlan(2, ring_transfers(2, 4, 1, 1, 100), link_cost={(0, 1): 0})


def test_route_shares_units_and_order():
    demand = {(0, a, (a + 1) % 6): 1000 for a in range(6)}
    shares, load = route_shares(6, demand, units=16, relay=True)
    for key, parts in shares.items():
        assert sum(n for _, n in parts) == 16
        paths = [k for k, _ in parts]
        assert paths == ([DIRECT] if DIRECT in paths else []) + sorted(k for k in paths if k != DIRECT)
        assert key[1] not in paths and key[2] not in paths


def test_slice_bounds_and_partition_shape():
    for P in (1, 63, 64, 1000, 25_000_000):
        for parts in (1, 2, 3, 8):
            b = slice_bounds(P, parts)
            assert b[0] == 0 and b[-1] == P and all(x <= y for x, y in zip(b, b[1:]))
            assert all(x % 64 == 0 or x == P for x in b[:-1])
    assert partition_shape("devices", 8, 128) == (8, 1)
    assert partition_shape("params", 8, 128) == (1, 8)
    assert partition_shape("hybrid", 8, 128, 2) == (2, 4)
    with pytest.raises(ValueError):
        partition_shape("hybrid", 8, 128, 3)
    with pytest.raises(ValueError):
        partition_shape("devices", 3, 128)


def _seeded(g, P):
    return torch.randn(P, generator=torch.Generator().manual_seed(7000 + g))


def _worker(rank, world, port, D, h, P, partition, gd, relay, staged, q, hr=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from oracle.cfa_oracle import sequential_mix
        shard, info = make_ring_shard(rank, world, D, h, h if hr is None else hr, P, "cpu", TorchTransport(), None,
                                      partition=partition, dev_groups=gd, relay=relay, staged=staged)
        lo, hi = info["slice"]
        plan = shard.plan
        for i in range(plan.L):
            shard.models[i] = _seeded(plan.first + i, P)[lo:hi]
        # every rank agrees on the schedule before running it
        digests = [None] * world
        dist.all_gather_object(digests, info.get("route_digest"))
        ok = len(set(digests)) == 1
        shard.exchange()

        def gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
        n, bad = shard.halo_check(gather, lo)  # every halo row equals its owner's (exact checksums)
        ok &= bad == 0 and n == ((plan.hl + plan.hr) if plan.world > 1 else 0)
        full = [_seeded(g, P).numpy() for g in range(D)]
        alphas = shard.alphas
        for i in range(plan.L):
            g = plan.first + i
            nb = plan.neighbours(g)
            srcs = [s.numpy() for s in shard.sources(i)]
            ok &= all(np.array_equal(s, full[j][lo:hi]) for s, j in zip(srcs, nb))
            got = sequential_mix(shard.models[i].numpy(), srcs, alphas)
            ref = sequential_mix(full[g], [full[j] for j in nb], alphas)[lo:hi]
            ok &= np.array_equal(got, ref)
        q.put((rank, bool(ok), info.get("route", {}).get("relay")))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,D,partition,gd,relay,staged", [
    (2, 16, "devices", None, True, True),
    (4, 16, "devices", None, False, True),
    (4, 32, "hybrid", 2, True, True),
    (8, 64, "devices", None, True, True),
    (8, 64, "devices", None, True, False),
    (8, 32, "hybrid", 4, True, True),
    (4, 16, "params", None, True, True),
])
def test_routed_exchange_gloo(world, D, partition, gd, relay, staged):
    """Multi-process (gloo) run of the strong-scaling round's exchange, checked against the
    unsharded population through the oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    P = 1000 + 37
    port = 31000 + (os.getpid() % 997) + world * 11 + D + (gd or 0) * 3 + int(relay) + 2 * int(staged)
    procs = [ctx.Process(target=_worker, args=(r, world, port, D, 4, P, partition, gd, relay, staged, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, used_relay = q.get(timeout=180)
        res[r] = ok
        if partition == "devices" and world == 8 and relay:
            assert used_relay
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def test_v4_ring_c5_shape_gloo():
    """Config 5's topology sharded as the driver's 8-GPU run would shard it: 128 devices on the
    TF2 v4 ring (N < 2: in-neighbour ii-1 only, consensus_v4.py:133-137, hl = 1, hr = 0) over 8
    ranks, routed exchange, every device's mix equal to the unsharded oracle's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, D, P = 8, 128, 515
    port = 32500 + (os.getpid() % 997)
    procs = [ctx.Process(target=_worker, args=(r, world, port, D, 1, P, "devices", None, True, True, q, 0))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, _ = q.get(timeout=180)
        res[r] = ok
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}
