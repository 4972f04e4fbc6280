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
        rates = _rates(world, 50.0, 50.0)
        shard, info = make_ring_shard(rank, world, D, 4, 4, P, "cpu", TorchTransport(), None, relay=True,
                                      partition=partition, dev_groups=gd,
                                      link_rates=rates, lane_token=tok[0], lane_agree=agree_gloo,
                                      lane_chunk_elems=256)
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


def _absent_peer_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import time

        from federated_amd.halo import Message
        from federated_amd.hostlane import HostLane, new_token
        from federated_amd.linkprobe import agree_gloo
        tok = [new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        bufs = {"send": torch.full((4096,), float(rank)), "recv": torch.zeros(4096)}
        msgs = [Message(0, a, 1 - a, "send", 0, "recv", 0, 4096, lane=True) for a in range(2)]
        lane = HostLane.open(rank, [m for m in msgs if m.src == rank], [m for m in msgs if m.dst == rank],
                             lambda k: bufs[k], "cpu", tok[0], agree_gloo, chunk_elems=1024, timeout_s=1.0)
        out = None
        if rank == 0:  # rank 1 never sends: rank 0's receive times out, loudly and boundedly
            t0 = time.monotonic()
            try:
                lane.run()
                out = "no error"
            except RuntimeError as exc:
                out = ("timeout" if "timed out" in str(exc) else str(exc), time.monotonic() - t0)
        agree_gloo(True)
        lane.close()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_absent_peer_times_out_loudly():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34100 + (os.getpid() % 997)
    procs = [ctx.Process(target=_absent_peer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    kind, seconds = res[0]
    assert kind == "timeout" and 0.9 < seconds < 10.0
