"""Per-link rates of the node the population is sharded over, measured before the routed halo is planned.

The reference has no collective (its neighbour models travel as files, TF1 ``cfa.py:119-130``);
the sharded population's only exchange is the ring halo of ``halo.py``, whose route plan needs a
cost per directed link. On one MI355X node every GPU has a direct xGMI link to each of the other
seven, but their rates are not given (the design's cost model assumed 50-64 GB/s per direction,
DESIGN.md §5): this module measures them with the same transport and message path the halo uses.

* ``matching_rounds``: a 1-factorisation of the ranks (round-robin "circle" schedule), so in each
  round every rank exchanges with exactly one partner and every link of the node is busy in both
  directions once over the rounds, while no GPU drives two links at a time.
* ``probe_links``: per round, each pair exchanges one ``elems``-float message each way, ``reps``
  times after a warm-up, timed with HIP events on the exchange stream (host clock on a
  host-staged transport); the pair's time is the slower end's. The same bytes are then sent as
  ``pieces`` messages in one group (the routed halo sends pieces of a row, not whole rows): the
  difference over the extra messages is the per-message cost. Then an all-peers pass: every rank
  sends to and receives from all peers at once (equal chunks), the per-GPU egress rate with every
  link busy together, which says whether the links of one GPU are independent (what the relayed
  routes assume).

Host logic (``matching_rounds``, ``rates_from_times``) is pure; ``probe_links`` runs on CPU tensors
over gloo as well (tests), and on the GPU over RCCL or torch.distributed (bench.py).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Tuple

ALIGN = 64


def matching_rounds(world: int) -> List[List[Tuple[int, int]]]:
    """Rounds of disjoint rank pairs covering every unordered pair exactly once (world - 1 rounds
    for an even world, world rounds with one rank idle per round for an odd one)."""
    if world < 2:
        return []
    n = world + (world % 2)
    ring = list(range(n))
    rounds = []
    for _ in range(n - 1):
        pairs = []
        for i in range(n // 2):
            a, b = ring[i], ring[n - 1 - i]
            if a < world and b < world:
                pairs.append((min(a, b), max(a, b)))
        rounds.append(sorted(pairs))
        ring = [ring[0], ring[-1]] + ring[1:-1]
    return rounds


def rates_from_times(times_s, elems: int, elem_bytes: int = 4) -> Dict[Tuple[int, int], float]:
    """Per-direction GB/s of every directed link from a [world][world] matrix of exchange times
    (seconds; entry [a][b] measured on rank a for its exchange with b, 0 = not measured): link a->b
    and b->a both take the slower end's time of their (bidirectional) exchange."""
    world = len(times_s)
    out = {}
    for a in range(world):
        for b in range(world):
            if a == b:
                continue
            t = max(float(times_s[a][b]), float(times_s[b][a]))
            if t > 0:
                out[(a, b)] = elems * elem_bytes / t / 1e9
    return out


def _prepare(transport, sends, recvs):
    prep = getattr(transport, "prepare", None)
    if prep is not None:
        return prep(sends, recvs)
    return lambda stream=None: transport.exchange(sends, recvs, stream)


def _timed(op, stream, reps: int, warmup: int, device_timing: bool) -> float:
    """Seconds per call of ``op(stream)``: HIP events around ``reps`` back-to-back calls on the
    stream (device transports), else the host clock with the stream drained on both sides."""
    import torch
    for _ in range(warmup):
        op(stream)
    if stream is not None:
        stream.synchronize()
    if device_timing:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            op(stream)
        b.record(stream)
        b.synchronize()
        return a.elapsed_time(b) / 1e3 / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        op(stream)
    if stream is not None:
        stream.synchronize()
    return (time.perf_counter() - t0) / reps


def probe_links(transport, rank: int, world: int, device=None, elems: int = 16 << 20, reps: int = 3,
                warmup: int = 1, all_peers: bool = True, group=None, pieces: int = 32) -> dict:
    """Measure every directed link (see the module docstring). Collective over the default
    torch.distributed group (``group``: another control group): every rank calls it with the same
    arguments. Returns {"rates": {(a, b): GB/s}, "pair_ms": [[ms]], "elems": elems,
    "pieces": {"count": pieces, "pair_ms": [[ms]]} or None,
    "all_peers": {"egress_GBps": [per rank], "chunk_elems": c} or None}, identical on every rank."""
    import torch
    import torch.distributed as dist

    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    elems = max(ALIGN, elems // ALIGN * ALIGN)
    send = torch.full((elems,), float(rank), dtype=torch.float32, device=dev)
    recv = torch.empty(elems, dtype=torch.float32, device=dev)
    if dev.type == "cuda":
        from .streams import role_stream
        stream = role_stream("comm", dev)  # the halo's own exchange stream (streams.py)
    else:
        stream = None
    device_timing = dev.type == "cuda" and not getattr(transport, "host_staged", False)
    times = torch.zeros((2, world, world), dtype=torch.float64)
    piece = max(ALIGN, elems // max(1, pieces) // ALIGN * ALIGN) if pieces > 1 else 0
    for pairs in matching_rounds(world):
        dist.barrier(group=group)  # one round at a time: no GPU drives two links
        partner = next((b if a == rank else a for a, b in pairs if rank in (a, b)), None)
        if partner is None:
            continue
        op = _prepare(transport, [(send, partner)], [(recv, partner)])
        times[0, rank, partner] = _timed(op, stream, reps, warmup, device_timing)
        if float(recv[0].item()) != float(partner):
            raise RuntimeError(f"link probe: rank {rank} received {float(recv[0].item())} from {partner}")
        if piece:
            k = elems // piece
            op = _prepare(transport, [(send[i * piece:(i + 1) * piece], partner) for i in range(k)],
                          [(recv[i * piece:(i + 1) * piece], partner) for i in range(k)])
            times[1, rank, partner] = _timed(op, stream, reps, warmup, device_timing) * elems / (k * piece)
    dist.all_reduce(times, op=dist.ReduceOp.SUM, group=group)  # each entry written by one rank
    t1, tp = times[0].tolist(), times[1].tolist()
    res = {"elems": elems, "rates": rates_from_times(t1, elems),
           "pair_ms": [[round(float(t) * 1e3, 4) for t in row] for row in t1], "all_peers": None,
           "pieces": {"count": elems // piece, "piece_elems": piece,
                      "pair_ms": [[round(float(t) * 1e3, 4) for t in row] for row in tp]} if piece else None}
    if all_peers and world > 2:
        chunk = max(ALIGN, elems // (world - 1) // ALIGN * ALIGN)
        peers = [p for p in range(world) if p != rank]
        sends = [(send[i * chunk:(i + 1) * chunk], p) for i, p in enumerate(peers)]
        recvs = [(recv[i * chunk:(i + 1) * chunk], p) for i, p in enumerate(peers)]
        dist.barrier(group=group)
        t = _timed(_prepare(transport, sends, recvs), stream, reps, warmup, device_timing)
        for i, p in enumerate(peers):
            if float(recv[i * chunk].item()) != float(p):
                raise RuntimeError(f"link probe (all peers): rank {rank} chunk {i} not from {p}")
        tv = torch.zeros(world, dtype=torch.float64)
        tv[rank] = t
        dist.all_reduce(tv, op=dist.ReduceOp.SUM, group=group)
        res["all_peers"] = {"chunk_elems": chunk,
                            "egress_GBps": [round((world - 1) * chunk * 4 / float(x) / 1e9, 2) if x > 0 else None
                                            for x in tv.tolist()]}
    del send, recv
    return res


def summarize(probe: dict, world: int) -> dict:
    """The bench line's view of a probe: the rate matrix (GB/s per direction, None on the
    diagonal), its min / median / max, and the all-peers egress against the sum of one GPU's
    pairwise link rates (1.0 = the links of a GPU add up; what relayed routes assume)."""
    import statistics
    rates = probe["rates"]
    mat = [[round(rates[(a, b)], 2) if (a, b) in rates else None for b in range(world)] for a in range(world)]
    vals = sorted(rates.values())
    out = {"message_MB": round(probe["elems"] * 4 / 1e6, 1), "rates_GBps": mat,
           "min_GBps": round(vals[0], 2) if vals else None,
           "median_GBps": round(statistics.median(vals), 2) if vals else None,
           "max_GBps": round(vals[-1], 2) if vals else None}
    pc = probe.get("pieces")
    if pc:
        # per-message cost: (time as `count` messages - time as one) / (count - 1), per pair
        extra = []
        for a in range(world):
            for b in range(a + 1, world):
                one = max(probe["pair_ms"][a][b], probe["pair_ms"][b][a])
                many = max(pc["pair_ms"][a][b], pc["pair_ms"][b][a])
                if one > 0 and many > 0 and pc["count"] > 1:
                    extra.append((many - one) / (pc["count"] - 1) * 1e3)
        out["pieces"] = {"count": pc["count"], "piece_MB": round(pc["piece_elems"] * 4 / 1e6, 2),
                         "per_message_us_median": round(statistics.median(extra), 2) if extra else None,
                         "pieces_rate_median_GBps": round(statistics.median(
                             [probe["elems"] * 4 / (max(pc["pair_ms"][a][b], pc["pair_ms"][b][a]) * 1e-3) / 1e9
                              for a in range(world) for b in range(a + 1, world)
                              if max(pc["pair_ms"][a][b], pc["pair_ms"][b][a]) > 0]), 2) if extra else None}
    ap = probe.get("all_peers")
    if ap:
        eg = ap["egress_GBps"]
        sums = [sum(rates.get((a, b), 0.0) for b in range(world) if b != a) for a in range(world)]
        out["all_peers_egress_GBps"] = eg
        out["all_peers_vs_link_sum"] = [round(e / s, 3) if (e and s) else None for e, s in zip(eg, sums)]
    return out


def min_rate(probe: Optional[dict]) -> Optional[float]:
    if not probe or not probe.get("rates"):
        return None
    return min(probe["rates"].values())


def agree_gloo(ok: bool, group=None) -> bool:
    """All-ranks AND over the control plane (a gloo all-reduce MIN): also a barrier."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def probe_lane(rank: int, world: int, device, token: str, agree=agree_gloo, elems: int = 64 << 20, reps: int = 3,
               warmup: int = 1, chunk_elems: Optional[int] = None, timeout_s: float = 60.0,
               numa_nodes=None, segment_elems: int = 0) -> dict:
    """The host lane's rates (``hostlane.py``) with every rank using it at once: rank a sends
    ``elems`` floats to rank a + 1 and receives as many from rank a - 1 over pinned shared host
    memory, D2H and H2D pipelined in chunks, ``reps`` timed rounds after ``warmup``: at world 2 the
    exact pattern of the N = 2 halo, and at any world every GPU's PCIe link busy in both
    directions while host memory serves all of them. Per rank: the out rate (its D2H stream's
    bytes / time) and the in rate (bytes / time from the first chunk's arrival in host memory to
    the last H2D: the pipelined lane's steady rate, free of the ranks' start skew; the planner
    adds the pipeline's fill separately), medians over the reps, HIP events on the lane's streams
    (host clock on CPU tensors). Collective (``agree(ok)``: the control plane's all-ranks AND; a failure
    on any rank raises on every rank). ``numa_nodes[r]``: rank r's GPU's NUMA node (segments are
    placed on the receiver's, as the headline's are); ``segment_elems``: reserve and pin segments
    of at least that many elements per parity (what the headline's plan may put on one pair), so
    that the probe fails where the headline's lane would. Returns {"rates":
    {(a, LANE_OUT): GB/s, (LANE_IN, b): GB/s}, "out_GBps": [per rank], "in_GBps": [per rank],
    "elems": elems, "chunk_elems": c, "pairs": [[a, a + 1] per rank], "numa_nodes"},
    identical on every rank (all-reduced)."""
    import statistics
    import torch
    import torch.distributed as dist
    from .halo import LANE_IN, LANE_OUT, Message
    from .hostlane import DEFAULT_CHUNK_ELEMS, HostLane

    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    elems = max(ALIGN, elems // ALIGN * ALIGN)
    bufs = {"send": torch.full((elems,), float(rank), dtype=torch.float32, device=dev),
            "recv": torch.empty(elems, dtype=torch.float32, device=dev)}
    msgs = [Message(0, a, (a + 1) % world, "send", 0, "recv", 0, elems, lane=True) for a in range(world)]
    lane = HostLane.open(rank, [m for m in msgs if m.src == rank], [m for m in msgs if m.dst == rank],
                         lambda k: bufs[k], dev, token, agree, chunk_elems=chunk_elems or DEFAULT_CHUNK_ELEMS,
                         timeout_s=timeout_s, numa_nodes=numa_nodes, segment_elems=segment_elems)
    gpu = dev.type == "cuda"
    stream = torch.cuda.current_stream(dev) if gpu else None
    outs, ins, err = [], [], None
    try:
        for _ in range(warmup):
            lane.run(stream)
            lane.finish()
        if gpu:
            torch.cuda.synchronize(dev)
        lane.check()
    except Exception as exc:
        err = f"{type(exc).__name__}: {exc}"
    if agree(err is None):
        # one agreement per rep, on every rank alike (the same number of collectives whatever
        # fails): each rep starts with every rank drained, so no ack wait or start skew is timed
        for _ in range(reps):
            try:
                t0 = time.perf_counter()
                lane.run(stream, timing=gpu)
                lane.finish()
                if gpu:
                    torch.cuda.synchronize(dev)
                    tm = lane.timing_ms()
                    outs.append(tm["out_ms"])
                    ins.append(tm.get("in_steady_ms", tm["in_ms"]))
                else:
                    dt = (time.perf_counter() - t0) * 1e3
                    outs.append(dt)
                    ins.append(dt)
                lane.check()
            except Exception as exc:
                err = f"{type(exc).__name__}: {exc}"
            if not agree(err is None):
                err = err or "a lane probe rep failed on another rank"
                break
        if err is None:
            src = (rank - 1) % world
            got = (float(bufs["recv"][0].item()), float(bufs["recv"][-1].item()))
            if got != (float(src), float(src)):
                err = f"lane probe: rank {rank} received {got}, not rank {src}'s rows"
    else:
        err = err or "the warm-up failed on another rank"
    lane.close()
    if not agree(err is None):
        raise RuntimeError(f"lane probe: {err or 'failed on another rank'}")
    t = torch.zeros((2, world), dtype=torch.float64)
    t[0, rank] = statistics.median(outs)
    t[1, rank] = statistics.median(ins)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    nbytes = elems * 4
    out_r = [nbytes / (float(x) * 1e-3) / 1e9 if x > 0 else 0.0 for x in t[0].tolist()]
    in_r = [nbytes / (float(x) * 1e-3) / 1e9 if x > 0 else 0.0 for x in t[1].tolist()]
    rates = {}
    for a in range(world):
        if out_r[a] > 0:
            rates[(a, LANE_OUT)] = out_r[a]
        if in_r[a] > 0:
            rates[(LANE_IN, a)] = in_r[a]
    del bufs
    return {"rates": rates, "out_GBps": [round(x, 2) for x in out_r], "in_GBps": [round(x, 2) for x in in_r],
            "elems": elems, "chunk_elems": lane.chunk_elems, "segment_elems": max(elems, int(segment_elems)),
            "pairs": [[a, (a + 1) % world] for a in range(world)],
            "numa_nodes": list(numa_nodes) if numa_nodes is not None else None,
            "timing": "HIP events on the lane streams" if gpu else "host clock (CPU tensors)"}


def lane_pair_rates(probe: dict, numa_nodes=None) -> dict:
    """The planner's lane rates from ``probe_lane``'s result, priced by pair where the GPUs sit on
    different NUMA nodes (a segment lives on its receiver's node, so a cross-node pair's D2H
    crosses the socket link):

    * a rank's pseudo-links (a, LANE_OUT) / (LANE_IN, a) take its probed rates, except that a
      rank whose probe pair was cross-node takes the median out rate of the same-node probe pairs
      (its own figure was the cross-socket one);
    * every cross-node directed pair (a, b) gets its own link (a, lane_pair(b)) at the slowest out
      rate the cross-node probe pairs measured.

    Without node information, or with every rank on one node, the probe's rates unchanged."""
    from .halo import LANE_OUT, lane_pair
    rates = dict(probe["rates"])
    nodes = list(numa_nodes) if numa_nodes is not None else probe.get("numa_nodes")
    world = len(probe.get("out_GBps") or [])
    if not nodes or world < 2 or len(nodes) < world or any(n is None or n < 0 for n in nodes[:world]):
        return rates
    cross = [a for a, b in probe.get("pairs", []) if nodes[a] != nodes[b]]
    if not cross:
        return rates
    same = [a for a, b in probe.get("pairs", []) if nodes[a] == nodes[b] and (a, LANE_OUT) in rates]
    x_rate = min(rates[(a, LANE_OUT)] for a in cross if (a, LANE_OUT) in rates)
    if same:
        import statistics
        local = statistics.median(rates[(a, LANE_OUT)] for a in same)
        for a in cross:
            if (a, LANE_OUT) in rates:
                rates[(a, LANE_OUT)] = local
    for a in range(world):
        for b in range(world):
            if a != b and nodes[a] != nodes[b]:
                rates[(a, lane_pair(b))] = x_rate
    return rates
