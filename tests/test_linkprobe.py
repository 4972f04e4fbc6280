"""CPU tests of the per-link probe (federated_amd/linkprobe.py) and of the round model the N > 1
bench line's decomposition reports (population.predict_round_ms).

- matching_rounds: every unordered rank pair exactly once, no rank twice in a round, for world
  sizes 2..9 (odd worlds leave one rank idle per round).
- probe_links over gloo at world 2 and 4 on CPU tensors (the bench's control-plane logic with
  the torch transport): every directed link gets a positive rate, the result is identical on every
  rank, and the all-peers pass reports one egress rate per rank.
- predict_round_ms: the exchange-bound and compute-bound cases and the contention stretch.
"""
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from federated_amd.linkprobe import matching_rounds, rates_from_times, summarize
from federated_amd.population import predict_round_ms


@pytest.mark.parametrize("world", range(1, 10))
def test_matching_rounds_cover_every_pair_once(world):
    rounds = matching_rounds(world)
    seen = []
    for pairs in rounds:
        ranks = [r for p in pairs for r in p]
        assert len(ranks) == len(set(ranks))  # a rank drives one link per round
        assert all(a < b < world for a, b in pairs)
        seen += pairs
    assert sorted(seen) == [(a, b) for a in range(world) for b in range(a + 1, world)]
    assert len(rounds) == (0 if world < 2 else world - 1 + world % 2)


def test_rates_take_the_slower_end():
    t = [[0.0, 0.002, 0.0], [0.004, 0.0, 0.001], [0.0, 0.001, 0.0]]
    r = rates_from_times(t, 1_000_000)
    assert r[(0, 1)] == r[(1, 0)] == pytest.approx(4e6 / 0.004 / 1e9)
    assert r[(1, 2)] == pytest.approx(4.0)
    assert (0, 2) not in r and (2, 0) not in r
    s = summarize({"elems": 1_000_000, "rates": r, "all_peers": None}, 3)
    assert s["rates_GBps"][0][0] is None and s["min_GBps"] == 1.0 and s["max_GBps"] == 4.0


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from federated_amd.linkprobe import probe_links
        res = probe_links(TorchTransport(), rank, world, None, elems=1 << 16, reps=2)
        q.put((rank, res, None))
    except Exception as exc:  # reported to the parent
        q.put((rank, None, repr(exc)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_probe_links_over_gloo(world):
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    errs = [e for _, _, e in out if e]
    assert not errs, errs
    results = {r: res for r, res, _ in out}
    first = results[0]
    assert set(first["rates"]) == {(a, b) for a in range(world) for b in range(world) if a != b}
    assert all(v > 0 for v in first["rates"].values())
    for res in results.values():  # identical on every rank (the route plan must be)
        assert res["rates"] == first["rates"] and res["pair_ms"] == first["pair_ms"]
    pc = first["pieces"]
    assert pc["count"] == 32 and all(pc["pair_ms"][a][b] > 0 for a in range(world) for b in range(world) if a != b)
    s2 = summarize(first, world)
    assert s2["pieces"]["count"] == 32 and s2["pieces"]["per_message_us_median"] is not None
    if world > 2:
        assert len(first["all_peers"]["egress_GBps"]) == world and all(first["all_peers"]["egress_GBps"])
        s = summarize(first, world)
        assert len(s["all_peers_vs_link_sum"]) == world
    else:
        assert first["all_peers"] is None


def test_round_model_exchange_bound():
    """Exchange of 3 groups x 2 ms; 2 interior mixes of 0.1 ms; boundary sets after groups 1 and 2:
    the round ends one tail of mixes after the last group."""
    t = predict_round_ms([2.0, 2.0, 2.0], [(1, 4), (2, 4)], 2, 0.1, 0.0)
    assert t == pytest.approx(6.0 + 4 * 0.1)


def test_round_model_compute_bound_and_contention():
    """Short exchange (0.5 ms), 20 interior mixes of 0.15 ms: compute-bound; while the exchange runs
    each mix takes (1 + delta) longer."""
    base = predict_round_ms([0.5], [(0, 2)], 20, 0.15, 0.0)
    assert base == pytest.approx(22 * 0.15)
    slow = predict_round_ms([0.5], [(0, 2)], 20, 0.15, 0.2)
    n_stretched = 3  # mixes started before t = 0.5 ms: at 0, 0.18, 0.36
    assert slow == pytest.approx(base + n_stretched * 0.15 * 0.2)


def test_round_model_without_exchange_is_the_mixes():
    assert predict_round_ms([], [], 5, 0.2, 0.5) == pytest.approx(1.0)


def test_round_model_waits_for_the_host_lane():
    """With the host lane a boundary set waits for both paths: here its lane pieces land at 7 ms,
    after its xGMI group (4 ms), so the set starts at 7 ms; the exchange lasts until the lane's
    end (8 ms), so mixes started before then are stretched; no lane pieces (None) = xGMI only."""
    t = predict_round_ms([2.0, 2.0], [(1, 4)], 2, 0.1, 0.0, lane_ready_ms=[7.0], lane_end_ms=8.0)
    assert t == pytest.approx(max(7.0 + 4 * 0.1, 8.0))
    t = predict_round_ms([2.0, 2.0], [(1, 4)], 2, 0.1, 0.0, lane_ready_ms=[None], lane_end_ms=0.0)
    assert t == pytest.approx(4.0 + 4 * 0.1)
    stretched = predict_round_ms([0.5], [(0, 2)], 20, 0.15, 0.2, lane_ready_ms=[0.2], lane_end_ms=1.0)
    assert stretched > predict_round_ms([0.5], [(0, 2)], 20, 0.15, 0.2)  # the lane keeps running past 0.5 ms
