"""CPU tests of the host lane (federated_amd/hostlane.py): routing part of the halo over PCIe
through shared pinned host memory, beside the xGMI links.

- Routing: the lane is offered only with measured lane rates; at N = 2 with equal rates it takes
  half the halo and halves the predicted exchange; lane pieces never reach the transport's message
  lists and pair up between sender and receiver; a slow lane is left out.
- Layout: both ends compute the same segment offsets and chunk lists from the plan.
- Protocol over gloo (world 2 and 4, real shared-memory segments, host copies instead of DMA):
  several rounds in a row (both buffer parities and the receiver's ack back-pressure), every halo
  row equal to the unsharded population's bucket, every mix equal to the oracle's; the segment
  names are gone once the lane is open; the lane probe returns a rate per rank and direction.
"""
import os
from collections import defaultdict

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from federated_amd.halo import (DIRECT, LANE, LANE_IN, LANE_OUT, RoutePlan, choose_route, is_lane_link,
                                ring_transfers, route_shares)
from federated_amd.hostlane import _reached, lane_chunks, lane_layout


def _rates(world, xgmi=50.0, lane=None):
    r = {(a, b): xgmi for a in range(world) for b in range(world) if a != b}
    if lane:
        r.update({(a, LANE_OUT): lane for a in range(world)})
        r.update({(LANE_IN, b): lane for b in range(world)})
    return r


def _check_lane_pairing(plan):
    for a in range(plan.world):
        sends, _ = plan.lane_ops(a)
        for b in range(plan.world):
            _, recvs = plan.lane_ops(b)
            assert [m for m in sends if m.dst == b] == [m for m in recvs if m.src == a]
    for g in range(len(plan.groups)):
        for r in range(plan.world):
            s, rv = plan.rank_ops(r, g)
            assert not any(m.lane for m in s + rv)
    for msgs in plan.groups:
        for m in msgs:
            if m.lane:  # direct: straight into the halo row, never a relay slot
                assert not (isinstance(m.dst_key, tuple) and m.dst_key[0] == "relay")
                assert m.src_off == m.dst_off and m.src_off % plan.align == 0


def test_lane_takes_half_the_n2_halo_at_equal_rates():
    tr = ring_transfers(2, 64, 4, 4, 25_000_000)
    rates = _rates(2, 50.0, 50.0)
    plan, rep = choose_route(2, tr, rates_gbps=rates, lane_chunk_bytes=16 << 20)
    assert rep["chosen"] == "uniform+lane" and rep["lane_offered"]
    assert plan.lane
    total = sum(t.hi - t.lo for t in tr)
    assert 0.45 * total <= plan.lane_elems() <= 0.55 * total
    base = RoutePlan(2, tr)
    assert plan.predicted_ms(rates) < 0.55 * base.predicted_ms(rates)
    _check_lane_pairing(plan)
    # pseudo-links in the per-group loads, not in the transport's message counts
    assert any(is_lane_link(l) for g in range(len(plan.groups)) for l in plan.group_link_elems(g))
    assert not any(is_lane_link(l) for g in range(len(plan.groups)) for l in plan.group_link_elems(g, lane=False))
    assert plan.digest() == RoutePlan(2, tr, lane=True).digest()


def test_lane_needs_measured_rates_and_is_dropped_when_slow():
    tr = ring_transfers(2, 64, 4, 4, 25_000_000)
    plan, rep = choose_route(2, tr, rates_gbps=_rates(2, 50.0))  # no lane rates: not offered
    assert not plan.lane and not rep["lane_offered"] and not any("+lane" in k for k in rep["candidates"])
    plan, rep = choose_route(2, tr, rates_gbps=None)
    assert not plan.lane
    # a lane at a twentieth of the link rate only adds its pipeline fill: not chosen
    plan, rep = choose_route(2, tr, rates_gbps=_rates(2, 50.0, 2.5), lane_chunk_bytes=16 << 20)
    assert not plan.lane and rep["chosen"] == "uniform"


@pytest.mark.parametrize("world", [4, 8])
def test_lane_with_relays_keeps_the_plan_invariants(world):
    from test_halo_route import _check_plan
    tr = ring_transfers(world, 128 // world, 4, 4, 25_000_000)
    rates = _rates(world, 50.0, 50.0)
    plan = RoutePlan(world, tr, relay=True, lane=True)
    _check_plan(plan)
    _check_lane_pairing(plan)
    assert plan.lane
    nolane = RoutePlan(world, tr, relay=True)
    assert plan.predicted_ms(rates) < nolane.predicted_ms(rates)
    # every rank's lane load sits on its own two pseudo-links
    out = defaultdict(int)
    for m in plan.lane_ops(0)[0]:
        out[m.dst] += m.count
    assert sum(out.values()) == plan.link_elems.get((0, LANE_OUT), 0)


def test_route_shares_orders_direct_lane_relays():
    demand = {(0, a, (a + 1) % 6): 1000 for a in range(6)}
    shares, load = route_shares(6, demand, units=16, relay=True, lane=True)
    for key, parts in shares.items():
        paths = [k for k, _ in parts]
        expect = ([DIRECT] if DIRECT in paths else []) + ([LANE] if LANE in paths else []) + \
            sorted(k for k in paths if k >= 0)
        assert paths == expect and sum(n for _, n in parts) == 16
    assert any(LANE in [k for k, _ in p] for p in shares.values())


def test_layout_and_chunks():
    from federated_amd.halo import Message
    msgs = [Message(0, 0, 1, ("models", 0), 0, ("left", 0), 0, 1000, lane=True),
            Message(1, 0, 1, ("models", 1), 64, ("left", 1), 64, 130, lane=True),
            Message(1, 0, 1, ("models", 2), 0, ("left", 2), 0, 64, lane=True)]
    offs, n = lane_layout(msgs)
    assert offs == [0, 1024, 1216] and n == 1280
    ch = lane_chunks(msgs, offs, 512, ramp=0)
    assert ch == [(0, 0, 512, 0), (0, 512, 488, 512), (1, 0, 130, 1024), (2, 0, 64, 1216)]
    # the default ramp: the round's first pieces 64, 128, 256 elements, then 512
    ch = lane_chunks(msgs, offs, 512)
    assert ch == [(0, 0, 64, 0), (0, 64, 128, 64), (0, 192, 256, 192), (0, 448, 512, 448), (0, 960, 40, 960),
                  (1, 0, 130, 1024), (2, 0, 64, 1216)]
    for ramp in (0, 3):
        ch = lane_chunks(msgs, offs, 512, ramp=ramp)
        for i, m in enumerate(msgs):  # every element of every message exactly once, in order
            pieces = [(lo, c) for j, lo, c, _ in ch if j == i]
            assert pieces[0][0] == 0 and sum(c for _, c in pieces) == m.count
            assert all(a[0] + a[1] == b[0] for a, b in zip(pieces, pieces[1:]))
            assert all(lo % 64 == 0 for lo, _ in pieces)


def test_sequence_order_wraps():
    assert _reached(5, 5) and _reached(6, 5) and not _reached(4, 5)
    assert _reached(2, 0xFFFFFFFE) and not _reached(0xFFFFFFFE, 2)


def _seeded(g, P):
    return torch.randn(P, generator=torch.Generator().manual_seed(9100 + g))


def _worker(rank, world, port, D, P, rounds, q, partition="devices", gd=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from federated_amd.hostlane import new_token
        from federated_amd.linkprobe import agree_gloo, probe_lane
        from federated_amd.population import make_ring_shard
        from oracle.cfa_oracle import sequential_mix
        tok = [new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        probe = probe_lane(rank, world, "cpu", tok[0] + "p", agree_gloo, elems=300_000, reps=2,
                           chunk_elems=64 * 1024)
        ok = set(probe["rates"]) == {(a, LANE_OUT) for a in range(world)} | {(LANE_IN, a) for a in range(world)}
        ok &= all(r > 0 for r in probe["rates"].values())
        from federated_amd.linkprobe import lane_pair_rates
        # a fake two-socket node: the first half of the ranks on NUMA node 0, the rest on node 1 (a
        # node this container may not have: the placement is then skipped, and said so)
        nodes = [0] * (world // 2) + [1] * (world - world // 2)
        pr = dict(probe, out_GBps=[50.0] * world, rates={k: 50.0 for k in probe["rates"]})
        rates = {**_rates(world, 50.0), **lane_pair_rates(pr, nodes)}
        shard, info = make_ring_shard(rank, world, D, 4, 4, P, "cpu", TorchTransport(), None, relay=True,
                                      partition=partition, dev_groups=gd,
                                      link_rates=rates, lane_token=tok[0], lane_agree=agree_gloo,
                                      lane_chunk_elems=256, lane_numa_nodes=nodes)
        pairs = info["lane"]["pairs"]
        ok &= all(p["src_node"] == nodes[rank] and p["dst_node"] == nodes[p["dst"]] for p in pairs)
        ok &= all(len(p["placed_nodes"]) >= 1 for p in pairs)
        ok &= bool(info["route"]["lane"]) and "+lane" in info["route_choice"]["chosen"]
        if partition == "devices":
            ok &= bool(info["route"]["relay"]) == (world == 8)  # at 8 ranks relays and the lane together
        lo, hi = info["slice"]
        agree_gloo(True)  # every rank has unlinked the names it created
        ok &= not [f for f in os.listdir("/dev/shm") if tok[0] in f]
        plan = shard.plan
        alphas = shard.alphas
        for r in range(rounds):
            for i in range(plan.L):
                shard.models[i] = (_seeded(plan.first + i, P) + r)[lo:hi]
            shard.exchange()
            full = [(_seeded(g, P) + r).numpy()[lo:hi] for g in range(D)]
            for i in range(plan.L):
                g = plan.first + i
                nb = plan.neighbours(g)
                srcs = [s.numpy() for s in shard.sources(i)]
                ok &= all(np.array_equal(s, full[j]) for s, j in zip(srcs, nb))
                got = sequential_mix(shard.models[i].numpy(), srcs, alphas)
                ok &= np.array_equal(got, sequential_mix(full[g], [full[j] for j in nb], alphas))
        def gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
        n, bad = shard.halo_check(gather, info["slice"][0])
        ok &= n == 8 and bad == 0
        shard.halo["left"][0][7] += 1.0  # one changed element is caught
        n, bad = shard.halo_check(gather, info["slice"][0])
        ok &= bad == 1
        lane_in = info["lane"]["in_MB"]
        shard.lane.close()
        q.put((rank, bool(ok), lane_in))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,D,partition,gd", [(2, 16, "devices", None), (4, 16, "devices", None),
                                                 (8, 64, "devices", None), (4, 16, "hybrid", 2)])
def test_host_lane_rounds_gloo(world, D, partition, gd):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    P = 5000 + 17
    port = 33500 + (os.getpid() % 997) + world * 7 + (gd or 0) * 3
    procs = [ctx.Process(target=_worker, args=(r, world, port, D, P, 4, q, partition, gd)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, lane_in = q.get(timeout=180)
        res[r] = ok
        assert lane_in > 0
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _absent_peer_worker(rank, world, port, q, stop_after):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import time

        from federated_amd.halo import Message
        from federated_amd.hostlane import HostLane, LaneTimeout, new_token
        from federated_amd.linkprobe import agree_gloo
        tok = [new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        bufs = {"send": torch.full((4096,), float(rank)), "recv": torch.zeros(4096)}
        msgs = [Message(0, a, 1 - a, "send", 0, "recv", 0, 4096, lane=True) for a in range(2)]
        lane = HostLane.open(rank, [m for m in msgs if m.src == rank], [m for m in msgs if m.dst == rank],
                             lambda k: bufs[k], "cpu", tok[0], agree_gloo, chunk_elems=1024, timeout_s=1.0)
        out = None
        if rank == 0:  # rank 1 stops sending after `stop_after` rounds: rank 0's NEXT round fails
            for r in range(stop_after):
                gates = lane.run()
                gates[0].wait()  # what a boundary set does before it mixes
                lane.finish()
                if not torch.equal(bufs["recv"], torch.full((4096,), 1.0 + r)):
                    out = f"round {r}: wrong rows"
            t0 = time.monotonic()
            try:
                gates = lane.run()  # the send side does not wait for rank 1 (two parities)
                gates[0].wait()     # the receive side does: this round raises, not the next
                out = out or "no error"
            except LaneTimeout as exc:
                out = out or ("timeout" if f"round {stop_after}:" in str(exc) else str(exc), time.monotonic() - t0)
            try:
                lane.run()
                refused = False
            except RuntimeError as exc:
                refused = f"round {stop_after}" in str(exc)
            out = (out, refused) if isinstance(out, tuple) else out
        else:
            for r in range(stop_after):
                bufs["send"].fill_(1.0 + r)
                lane.run()
                lane.finish()
        agree_gloo(True)
        lane.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("stop_after", [0, 3])
def test_absent_peer_fails_its_own_round_loudly(stop_after):
    """Host-side waits (round 6): a chunk that never comes raises LaneTimeout in the round it
    belongs to (the first round, or round 3 after three good ones), after about the lane's timeout,
    and the lane refuses every later round."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34100 + (os.getpid() % 997) + stop_after * 11
    procs = [ctx.Process(target=_absent_peer_worker, args=(r, 2, port, q, stop_after)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    (kind, seconds), refused = res[0]
    assert kind == "timeout" and 0.9 < seconds < 10.0
    assert refused


def test_two_socket_topology_sheds_cross_pairs():
    """A fake two-socket node (ranks 0-3 on node 0, 4-7 on node 1): the lane probe's ring pairs
    3 -> 4 and 7 -> 0 cross the socket link and measured 15 GB/s against 50 for the others.
    lane_pair_rates gives ranks 3 and 7 the same-node rate on their own pseudo-links and every
    cross-node pair a link of its own at 15 GB/s; choose_route then puts less on a cross-node
    pair's lane than on a same-node pair's, and predicts a shorter exchange than when it prices
    every pair at its sender's rate."""
    from federated_amd.halo import lane_pair, priced_pairs
    from federated_amd.linkprobe import lane_pair_rates
    world = 8
    nodes = [0, 0, 0, 0, 1, 1, 1, 1]
    out = [50.0] * world
    out[3] = out[7] = 15.0
    probe = {"rates": {**{(a, LANE_OUT): out[a] for a in range(world)}, **{(LANE_IN, a): 50.0 for a in range(world)}},
             "out_GBps": out, "in_GBps": [50.0] * world, "pairs": [[a, (a + 1) % world] for a in range(world)]}
    rates = lane_pair_rates(probe, nodes)
    assert rates[(3, LANE_OUT)] == 50.0 and rates[(7, LANE_OUT)] == 50.0
    assert rates[(3, lane_pair(4))] == 15.0 and rates[(0, lane_pair(7))] == 15.0 and (0, lane_pair(1)) not in rates
    assert priced_pairs(rates) == {(a, b) for a in range(8) for b in range(8) if nodes[a] != nodes[b]}
    assert lane_pair_rates(probe, [0] * world) == probe["rates"]  # one node: unchanged
    assert lane_pair_rates(probe, None) == probe["rates"]
    full = {**_rates(world, 50.0), **rates}
    tr = ring_transfers(world, 16, 4, 4, 25_000_000)
    plan, rep = choose_route(world, tr, rates_gbps=full, lane_chunk_bytes=4 << 20)
    assert plan.lane and rep["lane_pairs_priced"]
    per = plan.lane_pair_elems()
    cross = [per.get((a, b), 0) for a, b in [(3, 4), (4, 3), (7, 0), (0, 7)]]
    same = [per.get((a, (a + 1) % 8), 0) for a in (0, 1, 4, 5)] + [per.get((a, a - 1), 0) for a in (2, 1, 6, 5)]
    assert max(cross) < min(same), (cross, same)
    # the same probe priced per rank (round 5): ranks 3 and 7 slow on every pair
    naive = {**_rates(world, 50.0), **probe["rates"]}
    nplan, _ = choose_route(world, tr, rates_gbps=naive, lane_chunk_bytes=4 << 20)
    assert plan.predicted_ms(full) <= nplan.predicted_ms(full) + 1e-9
    _check_lane_pairing(plan)


def test_numa_helpers_degrade_instead_of_failing():
    """numa.py: the thread policy on a node this host has is applied and restored; on one it does
    not have (or with no node) the block still runs and says why; node_of reports a node for a
    touched page or None. A segment created for a missing node still works."""
    import mmap as _mmap
    import ctypes as _ct

    from federated_amd import numa
    with numa.preferred(0) as why:
        assert why is None or isinstance(why, str)
    with numa.preferred(None) as why:
        assert why == "no NUMA node given"
    with numa.preferred(1 << 12) as why:  # no such node
        assert isinstance(why, str) and "set_mempolicy" in why
    m = _mmap.mmap(-1, 1 << 16)
    m[0] = 1
    n = numa.node_of(_ct.addressof(_ct.c_char.from_buffer(m)))
    assert n is None or n >= 0
    from federated_amd.hostlane import _Segment
    path = f"/dev/shm/cfa_lane_test_numa_{os.getpid()}"
    seg = _Segment(path, 1024, create=True, numa_node=1 << 12)
    try:
        assert seg.numa_note and "set_mempolicy" in seg.numa_note
        seg.data[:4] = torch.arange(4.0)
        assert seg.data[:4].tolist() == [0.0, 1.0, 2.0, 3.0]
        assert len(seg.placed_nodes()) >= 1
    finally:
        os.unlink(path)
        seg.close()


def test_stream_roles_are_gpu_only_and_named():
    from federated_amd import streams
    with pytest.raises(ValueError, match="unknown stream role"):
        streams.role_stream("compute2", "cuda:0")
    with pytest.raises(ValueError, match="GPU streams"):
        streams.role_stream("comm", "cpu")
    assert isinstance(streams.budget(), dict)


def _fuzz_worker(rank, world, port, cases, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from federated_amd.hostlane import new_token
        from federated_amd.linkprobe import agree_gloo
        from federated_amd.population import make_ring_shard
        results = []
        for ci, (D, h, P, chunk, lane_rate, rounds) in enumerate(cases):
            tok = [new_token() if rank == 0 else None]
            dist.broadcast_object_list(tok, src=0)
            rates = _rates(world, 50.0, lane_rate)
            shard, info = make_ring_shard(rank, world, D, h, h, P, "cpu", TorchTransport(), None, relay=True,
                                          link_rates=rates, lane_token=tok[0], lane_agree=agree_gloo,
                                          lane_chunk_elems=chunk)
            ok = True
            for r in range(rounds):
                for i in range(shard.plan.L):
                    g = shard.plan.first + i
                    shard.models[i] = torch.randn(P, generator=torch.Generator().manual_seed(31 * g + 7 * r + ci))
                shard.exchange()
                for i in shard.plan.boundary():
                    g = shard.plan.first + i
                    for src, j in zip(shard.sources(i), shard.plan.neighbours(g)):
                        want = torch.randn(P, generator=torch.Generator().manual_seed(31 * j + 7 * r + ci))
                        ok &= torch.equal(src, want)
            results.append((ci, bool(ok), bool(info["route"]["lane"]), info["route"]["lane_elems"]))
            shard.close()
        q.put((rank, results))
    except Exception as exc:
        q.put((rank, f"{type(exc).__name__}: {exc}"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_lane_random_plans_gloo(world):
    """Random ring populations (devices, window, odd bucket lengths, chunk sizes from one aligned
    piece to several pieces per row, lane rates that give the lane anything from a sliver to most
    of the halo), three rounds each, with fresh models every round: every halo row any boundary
    device reads equals its owner's row of that round, on every rank."""
    import random
    rng = random.Random(4242 + world)
    cases = []
    for _ in range(5):
        h = rng.randint(1, 3)
        D = world * rng.randint(2 * h, 2 * h + 3)
        cases.append((D, h, rng.randint(300, 4000) * 3 + 1, 64 * rng.randint(1, 40), rng.choice([5.0, 25.0, 50.0, 200.0]),
                      3))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 35900 + (os.getpid() % 997) + world * 13
    procs = [ctx.Process(target=_fuzz_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, out = q.get(timeout=240)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
    for r, out in res.items():
        assert not isinstance(out, str), f"rank {r}: {out}"
        assert all(ok for _, ok, _, _ in out), (r, out)
    assert any(used for _, _, used, _ in res[0])  # the lane carried pieces in some of the plans


def test_pair_links_in_plan_loads_and_prices():
    """A priced lane pair loads its own pseudo-link beside the two rank links, in the plan's link
    loads and its predicted group time; unpriced pairs do not. lane_pair_rates leaves the rates
    alone with missing or partial node information."""
    from federated_amd.halo import lane_pair, lane_pair_dst, priced_pairs
    from federated_amd.linkprobe import lane_pair_rates
    assert lane_pair_dst(lane_pair(5)) == 5 and lane_pair_dst(LANE_OUT) is None and lane_pair_dst(LANE_IN) is None
    tr = ring_transfers(2, 16, 4, 4, 100_000)
    rates = _rates(2, 50.0, 50.0)
    rates[(0, lane_pair(1))] = 10.0  # only 0 -> 1 crosses sockets
    assert priced_pairs(rates) == {(0, 1)}
    plan = RoutePlan(2, tr, lane=True, lane_pairs=priced_pairs(rates))
    assert plan.lane
    loads = {}
    for g in range(len(plan.groups)):
        for l, n in plan.group_link_elems(g).items():
            loads[l] = loads.get(l, 0) + n
    per = plan.lane_pair_elems()
    assert loads.get((0, lane_pair(1)), 0) == per.get((0, 1), 0) > 0
    assert (1, lane_pair(0)) not in loads
    # the slow pair link sets the price of groups that carry 0 -> 1 lane pieces
    fast = plan.predicted_ms({k: v for k, v in rates.items() if k != (0, lane_pair(1))})
    assert plan.predicted_ms(rates) > fast
    probe = {"rates": {(0, LANE_OUT): 50.0, (1, LANE_OUT): 20.0, (LANE_IN, 0): 50.0, (LANE_IN, 1): 50.0},
             "out_GBps": [50.0, 20.0], "pairs": [[0, 1], [1, 0]]}
    assert lane_pair_rates(probe, [0, None]) == probe["rates"]  # a node unknown: unchanged
    assert lane_pair_rates(probe, [0]) == probe["rates"]        # too short: unchanged
    both_cross = lane_pair_rates(probe, [0, 1])                  # no same-node probe pair: ranks keep theirs
    assert both_cross[(1, LANE_OUT)] == 20.0 and both_cross[(0, lane_pair(1))] == 20.0
