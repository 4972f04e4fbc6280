"""Routed halo exchange for a population sharded over the GPUs of one fully connected xGMI node.

The reference has no collective at all: a simulated device reads each neighbour's published
model from a shared directory (TF1 ``cfa.py:119-130``, TF2 ``consensus_v3.py:82-141``). When the
population is sharded in contiguous device blocks (SURVEY §8 e), a round's only cross-shard
traffic is the boundary buckets each rank's devices read from the neighbouring ranks. On a ring
window that is h buckets from each side, always to the SAME two peers, so sent directly the
whole halo rides two of the seven xGMI links of a GPU while five idle. Under strong scaling (a
fixed population over more GPUs) the halo stays 2h buckets per rank while the mixing work
shrinks as 1/N, so the two links become the round's critical path.

This module spreads the halo over every link:

* **Routing** (``route_shares``). The demand between each ordered rank pair (a, b) is split in
  ``units`` equal parts (64 by default: the bench's N = 8 relayed plan's critical path is 206.3 MB
  against 212.5 MB with 32 parts and 218.8 MB with 16; consecutive parts on one path merge into
  one message, so the message count stays the same). Each part goes direct (link a->b) or is relayed through a third rank k
  (links a->k, k->b). A greedy pass assigns the parts one at a time to the path whose busier link
  ends up least loaded. It is integer arithmetic with a fixed tie-break, so every rank computes
  the same routes without talking (and ``RoutePlan.digest`` lets the caller check that).
* **Stages.** Transfers carry a stage index: the bench's ring plan sends the rows the most
  boundary devices need first, so those devices can mix while later rows are still in flight.
* **Groups.** A relayed piece needs two hops, and the second may only start once the first has
  landed. Group g holds the direct pieces and first hops of stage g plus the second hops of
  stage g - 1, so groups run back to back on one stream and every link stays busy. Stage s is
  complete after group s + 1 (after group s when nothing is relayed). A relay rank keeps the
  pieces in two staging slots, by stage parity.
* **Measured links** (``link_cost``). By default every link costs the same per element. Given
  integer costs per directed link (``link_costs_from_rates`` of the rates ``linkprobe`` measures
  on the node), a part's weight on a link is its elements times that link's cost, so the greedy
  moves parts off slow links and the critical path is in time units; ``predicted_ms`` turns a
  plan back into milliseconds with the measured rates.
* **Host lane** (``lane=True``, ``hostlane.py``). A third kind of path: the piece goes D2H over
  the sender's PCIe link into shared pinned host memory and H2D over the receiver's, beside the
  xGMI links. In the load model the lane is two pseudo-links per rank, ``(a, LANE_OUT)`` (a's D2H)
  and ``(LANE_IN, b)`` (b's H2D), each shared by all of that rank's lane pieces; with measured
  rates for them (``linkprobe.probe_lane``) the greedy puts on the lane what shortens the critical
  path. Lane messages never reach the transport (``rank_ops`` leaves them out; ``lane_ops`` lists
  them). A pair whose two GPUs sit on different NUMA nodes (``numa.py``) also has a rate of its
  own: the pseudo-link ``(a, lane_pair(b))``, loaded only by that pair's lane pieces, priced at the
  probed cross-socket rate (``linkprobe.lane_pair_rates``), so the greedy sheds lane pieces from
  cross-socket pairs first.
* **Messages.** Each piece is one contiguous element range, so a message is one RCCL
  send/recv of a plain buffer slice. Within a group, every rank lists its sends to a peer in the
  order of one global message list, and the peer lists its receives in that same order, so the
  k-th send pairs with the k-th receive (RCCL matches point-to-point operations between a rank
  pair in issue order).

Nothing here touches a GPU: ``RoutePlan`` is pure host logic (tested on CPU, with gloo at world
sizes up to 8); ``RoutedExchange`` binds a plan to one rank's buffers and a transport.
"""
from __future__ import annotations

import hashlib
from collections import defaultdict
from dataclasses import dataclass
from typing import Callable, Dict, Hashable, List, Optional, Sequence, Tuple

ALIGN = 64  # elements: every piece starts 256-byte aligned (float4 kernels, RCCL copies)
DIRECT = -1
LANE = -2      # path id of the host lane
LANE_OUT = -2  # pseudo endpoints of the lane in link keys: (a, LANE_OUT) is rank a's D2H,
LANE_IN = -3   # (LANE_IN, b) is rank b's H2D
LANE_PAIR = -16  # (a, LANE_PAIR - b): the lane path of pair a -> b alone (priced pairs only)


def is_lane_link(link: Tuple[int, int]) -> bool:
    """Is a directed link key one of the host lane's pseudo-links?"""
    return link[0] < 0 or link[1] < 0


def lane_pair(b: int) -> int:
    """The pseudo endpoint of pair (a, b)'s own lane link: key (a, lane_pair(b))."""
    return LANE_PAIR - int(b)


def lane_pair_dst(e: int) -> Optional[int]:
    """b for a pair endpoint lane_pair(b), else None."""
    return LANE_PAIR - e if e <= LANE_PAIR else None


def priced_pairs(keys) -> frozenset:
    """The (a, b) pairs that have a lane pair link among ``keys`` (a cost or rate dict's keys)."""
    return frozenset((a, lane_pair_dst(e)) for a, e in keys if a >= 0 and lane_pair_dst(e) is not None)


def path_links(g: int, a: int, b: int, k: int, pairs: frozenset = frozenset()) -> List[Tuple[int, int, int]]:
    """The (group, from, to) links a piece of demand (g, a, b) loads on path k: the direct link;
    the lane's two pseudo-links (same group: the lane streams are not ordered behind the groups),
    plus the pair's own lane link when (a, b) is in ``pairs``; or relay k's first hop in group g
    and second hop in group g + 1."""
    if k == DIRECT:
        return [(g, a, b)]
    if k == LANE:
        return [(g, a, LANE_OUT), (g, LANE_IN, b)] + ([(g, a, lane_pair(b))] if (a, b) in pairs else [])
    return [(g, a, k), (g + 1, k, b)]


@dataclass(frozen=True)
class Transfer:
    """Move elements [lo, hi) of bucket ``src_key`` on rank ``src`` to the same range of bucket
    ``dst_key`` on rank ``dst``, as part of ``stage``."""
    stage: int
    src: int
    dst: int
    src_key: Hashable
    dst_key: Hashable
    lo: int
    hi: int


@dataclass(frozen=True)
class Message:
    """One point-to-point send/recv of ``count`` contiguous elements."""
    group: int
    src: int
    dst: int
    src_key: Hashable
    src_off: int
    dst_key: Hashable
    dst_off: int
    count: int
    lane: bool = False  # carried by the host lane (hostlane.py), not the transport


def relay_key(parity: int) -> tuple:
    return ("relay", parity)


def route_shares(world: int, demand: Dict[Tuple[int, int, int], int], units: int = 64,
                 relay: bool = True, cost: Optional[Dict[Tuple[int, int], int]] = None,
                 lane: bool = False) -> Tuple[Dict[Tuple[int, int, int], List[Tuple[int, int]]], Dict]:
    """Split every (group, a, b) demand over the direct link and 2-hop relays.

    ``demand[(g, a, b)]`` is the weight (elements) rank a sends rank b in stage position g. A
    direct piece loads link a->b in group g; a relayed piece loads a->k in group g and k->b in
    group g + 1. Parts are assigned one at a time, stage by stage, to the path that adds least to
    the exchange's critical path (the sum over groups of the busiest link's load, groups running
    back to back), then to the path whose busiest link ends up least loaded, then to fewer hops,
    then to the lower relay rank: integer arithmetic with a fixed order, so every rank computes
    the same routes. ``cost[(a, b)]`` (positive integers, default 1 for every link) scales a
    part's weight on link a->b: with costs proportional to 1 / measured rate the loads are times.
    ``lane`` adds the host lane (path LANE: pseudo-links (a, LANE_OUT) and (LANE_IN, b), and the
    pair link (a, lane_pair(b)) when ``cost`` has one; costs from ``cost`` like any link). Returns ``shares[(g, a, b)]`` = [(path, n_units)], path =
    DIRECT, LANE or the relay rank, direct first, then the lane, then relays ascending, n_units
    summing to ``units``; and the link loads per group, ``{(g, a, b): weight}``."""
    c = (lambda a, b: 1) if not cost else (lambda a, b: int(cost.get((a, b), 1)))
    pairs = priced_pairs(cost or {})
    load: Dict[Tuple[int, int, int], int] = defaultdict(int)
    gmax: Dict[int, int] = defaultdict(int)
    counts = {key: defaultdict(int) for key in demand}
    keys = sorted(k for k in demand if demand[k] > 0)
    for g in sorted({k[0] for k in keys}):
        stage_keys = [k for k in keys if k[0] == g]
        for _ in range(units):
            for key in stage_keys:
                _, a, b = key
                w = (demand[key] + units - 1) // units
                best, best_cost = DIRECT, None
                cands = [DIRECT] + ([LANE] if lane else []) + \
                    ([k for k in range(world) if k != a and k != b] if relay else [])
                for k in cands:
                    links = path_links(g, a, b, k, pairs)
                    delta = sum(max(0, load[l] + w * c(l[1], l[2]) - gmax[l[0]]) for l in links)
                    key_cost = (delta, max(load[l] + w * c(l[1], l[2]) for l in links), len(links), k)
                    if best_cost is None or key_cost < best_cost:
                        best, best_cost = k, key_cost
                for l in path_links(g, a, b, best, pairs):
                    load[l] += w * c(l[1], l[2])
                    gmax[l[0]] = max(gmax[l[0]], load[l])
                counts[key][best] += 1
    shares = {}
    for key in demand:
        c = counts[key]
        order = ([DIRECT] if c.get(DIRECT) else []) + ([LANE] if c.get(LANE) else []) + \
            sorted(k for k in c if k >= 0 and c[k])
        shares[key] = [(k, c[k]) for k in order]
    return shares, dict(load)


def _critical(shares, demand, cost=None) -> int:
    """Sum over groups of the busiest link's (cost-weighted) load for a set of shares."""
    load: Dict[Tuple[int, int, int], int] = defaultdict(int)
    pairs = priced_pairs(cost or {})
    for (g, a, b), parts in shares.items():
        units = sum(n for _, n in parts) or 1
        for k, n in parts:
            w = demand[(g, a, b)] * n // units
            for l in path_links(g, a, b, k, pairs):
                load[l] += w * (int(cost.get((l[1], l[2]), 1)) if cost else 1)
    gmax: Dict[int, int] = defaultdict(int)
    for (g, _, _), w in load.items():
        gmax[g] = max(gmax[g], w)
    return sum(gmax.values())


def _cuts(lo: int, hi: int, units: int, align: int) -> List[int]:
    """units + 1 aligned cut points from lo to hi (first lo, last hi)."""
    n = hi - lo
    pts = [lo]
    for u in range(1, units):
        x = lo + (n * u // units) // align * align
        pts.append(min(max(x, pts[-1]), hi))
    pts.append(hi)
    return pts


class RoutePlan:
    """The global message schedule of one routed exchange (identical on every rank)."""

    def __init__(self, world: int, transfers: Sequence[Transfer], relay: bool = True, units: int = 64,
                 align: int = ALIGN, link_cost: Optional[Dict[Tuple[int, int], int]] = None,
                 lane: bool = False, lane_pairs=None):
        """``link_cost``: integer cost per element of each directed link (``link_costs_from_rates``;
        the lane's pseudo-links included when ``lane``); None = every link alike. ``lane`` offers
        the host lane as a path (kept only where it shortens the critical path). ``lane_pairs``:
        the (a, b) pairs whose lane pieces also load their own pair link (cross-socket pairs with
        a probed rate; default: the pairs ``link_cost`` prices). Every rank must pass the same
        costs (the digest covers the routes they produce)."""
        self.world = int(world)
        self.link_cost = {k: int(v) for k, v in link_cost.items()} if link_cost else None
        self.lane_pairs = frozenset(lane_pairs) if lane_pairs is not None else priced_pairs(self.link_cost or {})
        for k, v in (self.link_cost or {}).items():
            if v < 1:
                raise ValueError(f"link cost must be a positive integer, got {k}: {v}")
        self.transfers = list(transfers)
        self.units, self.align = int(units), int(align)
        for t in self.transfers:
            if not (0 <= t.src < world and 0 <= t.dst < world) or t.src == t.dst or t.hi < t.lo:
                raise ValueError(f"bad transfer {t}")
        self.stages = sorted({t.stage for t in self.transfers})
        self._stage_pos = {s: i for i, s in enumerate(self.stages)}
        demand: Dict[Tuple[int, int, int], int] = defaultdict(int)
        for t in self.transfers:
            demand[(self._stage_pos[t.stage], t.src, t.dst)] += t.hi - t.lo
        self.relay = bool(relay) and world >= 3
        self.lane = bool(lane)
        lc = self.link_cost
        self.shares, _ = route_shares(world, dict(demand), self.units, self.relay, lc, self.lane)
        self.relay_considered = self.relay
        if self.relay:  # keep relays only where they shorten the (cost-weighted) critical path
            direct, _ = route_shares(world, dict(demand), self.units, False, lc, self.lane)
            if _critical(direct, dict(demand), lc) <= _critical(self.shares, dict(demand), lc):
                self.relay, self.shares = False, direct
        if self.lane:  # likewise the lane
            nolane, _ = route_shares(world, dict(demand), self.units, self.relay, lc, False)
            if _critical(nolane, dict(demand), lc) <= _critical(self.shares, dict(demand), lc):
                self.lane, self.shares = False, nolane
        self.groups: List[List[Message]] = [[] for _ in range(len(self.stages) + (1 if self.relay else 0))]
        slot_use = defaultdict(int)  # (rank, stage) -> relay elements
        self.link_elems: Dict[Tuple[int, int], int] = defaultdict(int)
        for t in self.transfers:
            g = self._stage_pos[t.stage]
            cuts = _cuts(t.lo, t.hi, self.units, self.align)
            u = 0
            for k, n in self.shares[(g, t.src, t.dst)]:
                x0, x1 = cuts[u], cuts[u + n]
                u += n
                cnt = x1 - x0
                if cnt <= 0:
                    continue
                if k == DIRECT:
                    self.groups[g].append(Message(g, t.src, t.dst, t.src_key, x0, t.dst_key, x0, cnt))
                    self.link_elems[(t.src, t.dst)] += cnt
                    continue
                if k == LANE:
                    self.groups[g].append(Message(g, t.src, t.dst, t.src_key, x0, t.dst_key, x0, cnt, lane=True))
                    self.link_elems[(t.src, LANE_OUT)] += cnt
                    self.link_elems[(LANE_IN, t.dst)] += cnt
                    if (t.src, t.dst) in self.lane_pairs:
                        self.link_elems[(t.src, lane_pair(t.dst))] += cnt
                    continue
                off = slot_use[(k, t.stage)]
                slot_use[(k, t.stage)] = off + -(-cnt // self.align) * self.align
                rk = relay_key(g % 2)
                self.groups[g].append(Message(g, t.src, k, t.src_key, x0, rk, off, cnt))
                self.groups[g + 1].append(Message(g + 1, k, t.dst, rk, off, t.dst_key, x0, cnt))
                self.link_elems[(t.src, k)] += cnt
                self.link_elems[(k, t.dst)] += cnt
        self._slot = defaultdict(int)
        for (k, _), n in slot_use.items():
            self._slot[k] = max(self._slot[k], n)
        while self.groups and not self.groups[-1]:
            self.groups.pop()

    # -- queries ---------------------------------------------------------------------------
    def slot_elems(self, rank: int) -> int:
        """Elements of one relay staging slot on ``rank`` (two slots are needed)."""
        return self._slot.get(rank, 0)

    def done_group(self, stage: int) -> int:
        """Index of the group after which every piece of ``stage`` has landed."""
        g = self._stage_pos[stage]
        return min(g + 1, len(self.groups) - 1) if self.relay else g

    def stages_done_after(self, group: int) -> List[int]:
        return [s for s in self.stages if self.done_group(s) == group]

    def rank_ops(self, rank: int, group: int) -> Tuple[List[Message], List[Message]]:
        """(sends, recvs) of ``rank`` in ``group`` over the transport, each in global message order
        (host-lane messages excluded: ``lane_ops``)."""
        msgs = [m for m in self.groups[group] if not m.lane]
        return [m for m in msgs if m.src == rank], [m for m in msgs if m.dst == rank]

    def lane_ops(self, rank: int) -> Tuple[List[Message], List[Message]]:
        """(sends, recvs) of ``rank`` over the host lane, every group, in global message order."""
        msgs = [m for g in self.groups for m in g if m.lane]
        return [m for m in msgs if m.src == rank], [m for m in msgs if m.dst == rank]

    def lane_elems(self) -> int:
        return sum(m.count for g in self.groups for m in g if m.lane)

    def lane_pair_elems(self) -> Dict[Tuple[int, int], int]:
        """Lane elements per (sender, receiver) pair."""
        out: Dict[Tuple[int, int], int] = defaultdict(int)
        for g in self.groups:
            for m in g:
                if m.lane:
                    out[(m.src, m.dst)] += m.count
        return dict(out)

    def max_link_elems(self) -> int:
        return max(self.link_elems.values(), default=0)

    def group_link_elems(self, group: int, lane: bool = True) -> Dict[Tuple[int, int], int]:
        """Elements per directed link in ``group``; the lane's pseudo-links included unless
        ``lane`` is False (the xGMI links alone)."""
        load: Dict[Tuple[int, int], int] = defaultdict(int)
        for m in self.groups[group]:
            if not m.lane:
                load[(m.src, m.dst)] += m.count
            elif lane:
                load[(m.src, LANE_OUT)] += m.count
                load[(LANE_IN, m.dst)] += m.count
                if (m.src, m.dst) in self.lane_pairs:
                    load[(m.src, lane_pair(m.dst))] += m.count
        return dict(load)

    def critical_elems(self) -> int:
        """Sum over groups of the busiest link's elements: the exchange time in units of
        elements per link-second when groups run back to back."""
        return sum(max(self.group_link_elems(g).values(), default=0) for g in range(len(self.groups)))

    def critical_cost(self) -> int:
        """Sum over groups of the busiest link's elements times that link's cost (= critical_elems
        when every link costs the same)."""
        total = 0
        for g in range(len(self.groups)):
            load = self.group_link_elems(g)
            total += max((n * (self.link_cost.get(l, 1) if self.link_cost else 1) for l, n in load.items()),
                         default=0)
        return total

    def max_rank_messages(self, group: int) -> int:
        """The most transport messages one rank issues in one direction (sends or receives) in
        ``group``."""
        sends: Dict[int, int] = defaultdict(int)
        recvs: Dict[int, int] = defaultdict(int)
        for m in self.groups[group]:
            if m.lane:
                continue
            sends[m.src] += 1
            recvs[m.dst] += 1
        return max(list(sends.values()) + list(recvs.values()), default=0)

    def predicted_group_ms(self, rates_gbps: Dict[Tuple[int, int], float], elem_bytes: int = 4,
                           message_us: float = 0.0) -> List[float]:
        """Per group, the time its slowest link needs at the given per-direction rates (GB/s; a link
        missing from ``rates_gbps`` takes the slowest rate given; the lane's pseudo-links take
        their probed rates), plus ``message_us`` per message of the rank that issues the most in the
        group (the per-message cost the link probe measures): the group's length when every link
        runs at its measured rate and the groups run back to back."""
        slow = min(rates_gbps.values()) if rates_gbps else None
        out = []
        for g in range(len(self.groups)):
            t = 0.0
            for l, n in self.group_link_elems(g).items():
                r = rates_gbps.get(l, slow)
                if r:
                    t = max(t, n * elem_bytes / (r * 1e9) * 1e3)
            if message_us > 0:
                t += message_us * 1e-3 * self.max_rank_messages(g)
            out.append(t)
        return out

    def predicted_ms(self, rates_gbps: Dict[Tuple[int, int], float], elem_bytes: int = 4,
                     message_us: float = 0.0, lane_chunk_bytes: int = 0) -> float:
        """Sum of ``predicted_group_ms``; with lane messages, plus the lane pipeline's fill: the
        first chunk (``lane_chunk_bytes``, ``hostlane.first_chunk_elems``) D2H before the first
        H2D can start, at the slowest lane rate."""
        t = sum(self.predicted_group_ms(rates_gbps, elem_bytes, message_us))
        if lane_chunk_bytes and any(m.lane for g in self.groups for m in g):
            lane_rates = [r for l, r in rates_gbps.items() if is_lane_link(l) and r > 0]
            if lane_rates:
                t += lane_chunk_bytes / (min(lane_rates) * 1e9) * 1e3
        return t

    def digest(self) -> str:
        h = hashlib.sha1()
        for g in self.groups:
            for m in g:
                h.update(repr(m).encode())
        return h.hexdigest()

    def summary(self) -> dict:
        return {
            "world": self.world, "relay": self.relay, "units": self.units,
            "groups": len(self.groups), "stages": len(self.stages),
            "messages": sum(len(g) for g in self.groups),
            "max_messages_per_rank_group": max(
                (len(s) + len(r) for g in range(len(self.groups)) for s, r in
                 [self.rank_ops(x, g) for x in range(self.world)]), default=0),
            "max_link_elems": self.max_link_elems(),
            "critical_elems": self.critical_elems(),
            "link_cost": "measured" if self.link_cost else "uniform",
            "lane": self.lane,
            "lane_elems": self.lane_elems(),
        }


class RoutedExchange:
    """A RoutePlan bound to one rank's buffers and a transport.

    ``buffers(key)`` returns the rank's 1-D tensor for a bucket key (the element ranges of the
    plan index into it). Relay staging is allocated here. ``run`` issues the groups in order on
    ``stream`` and calls ``stage_done(stage)`` right after the group that completes each stage,
    so the caller can record an event there and start that stage's boundary mixes. A plan with
    host-lane messages needs ``lane`` (a ``hostlane.HostLane`` opened on the same plan): ``run``
    starts its round first (the D2H side on the lane's own stream, the receive side on its pump
    thread), and ``lane_event(stage)`` is the gate a stream waits on for the lane's pieces of that
    stage (and every earlier one); ``finish_lane`` completes the lane's round on the host."""

    def __init__(self, plan: RoutePlan, rank: int, buffers: Callable[[Hashable], "object"], transport,
                 device=None, dtype=None, relay=None, lane=None):
        """``relay``: caller-provided staging of shape ``[2, >= slot_elems(rank)]`` (e.g. carved from
        a calibrated allocation); allocated here when None."""
        import torch
        self.plan, self.rank, self.transport = plan, int(rank), transport
        ls, lr = plan.lane_ops(self.rank)
        if (ls or lr) and lane is None:
            raise ValueError(f"rank {rank}: the plan sends {len(ls)} / receives {len(lr)} pieces over the host lane "
                             "but no lane was opened (population.RingPopulationShard.open_lane)")
        self.lane = lane
        self._lane_events = {}
        n = plan.slot_elems(self.rank)
        if relay is not None:
            if relay.dim() != 2 or relay.shape[0] != 2 or relay.shape[1] < n:
                raise ValueError(f"relay staging must be [2, >= {n}]")
            self.relay = relay
        else:
            self.relay = torch.empty((2, max(n, 1)), dtype=dtype or torch.float32, device=device)

        def view(key, off, cnt):
            buf = self.relay[key[1]] if isinstance(key, tuple) and key and key[0] == "relay" else buffers(key)
            return buf.reshape(-1)[off:off + cnt]

        self.ops = []
        for g in range(len(plan.groups)):
            sends, recvs = plan.rank_ops(self.rank, g)
            s = [(view(m.src_key, m.src_off, m.count), m.dst) for m in sends]
            r = [(view(m.dst_key, m.dst_off, m.count), m.src) for m in recvs]
            prep = getattr(transport, "prepare", None)
            self.ops.append(prep(s, r) if prep is not None else (s, r))
        self.done = [plan.stages_done_after(g) for g in range(len(plan.groups))]

    def lane_event(self, stage: int):
        """The lane gate (``hostlane.LaneGate``: ``stream.wait_event(gate)`` pumps the lane on the
        host until its pieces are enqueued, then waits for them) of the last group at or before
        ``stage``'s group (None: nothing of it on the lane)."""
        pos = self.plan.stages.index(stage)
        best = None
        for g, e in self._lane_events.items():
            if g <= pos and (best is None or g > best[0]):
                best = (g, e)
        return best[1] if best else None

    def run(self, stream=None, stage_done: Optional[Callable[[int], None]] = None,
            group_done: Optional[Callable[[int], None]] = None, lane_timing: bool = False,
            before_groups: Optional[Callable[[], None]] = None) -> None:
        """Issue every group in order; ``group_done(g)`` (optional) right after group g is issued
        (the bench's exchange-only timing records an event there). The host lane's copies go first,
        on its own streams after ``stream``'s earlier work (``lane_timing``: with HIP events);
        ``before_groups()`` (optional) runs after them and before the first group (the round's
        interior mixes, when the transport blocks the host)."""
        if self.lane is not None:
            self._lane_events = self.lane.run(stream, timing=lane_timing)
        if before_groups is not None:
            before_groups()
        for g, op in enumerate(self.ops):
            if self.lane is not None:
                self.lane.pump()
            if callable(op):
                op(stream)
            else:
                self.transport.exchange(op[0], op[1], stream)
            if group_done is not None:
                group_done(g)
            if stage_done is not None:
                for s in self.done[g]:
                    stage_done(s)

    def finish_lane(self) -> None:
        """Complete the round's host-lane part on the host (every H2D enqueued, ACKs raised); a
        no-op without a lane. ``population`` calls it through ``wait_streams`` at the round's end."""
        if self.lane is not None:
            self.lane.finish()


def link_costs_from_rates(rates_gbps: Dict[Tuple[int, int], float], scale: int = 16,
                          tolerance: float = 0.15) -> Dict[Tuple[int, int], int]:
    """Integer per-element cost of each directed link from measured rates. Links within
    ``tolerance`` of the median rate (or faster) cost ``scale``: the probe's run-to-run noise must
    not reshape a plan that is optimal for equal links. A slower link costs scale * median / rate
    (rounded): a link at half the median rate costs 2 * scale. Integer so that every rank plans the
    same routes from the same (all-reduced) rates."""
    if not rates_gbps:
        return {}
    vals = sorted(rates_gbps.values())
    for l, r in rates_gbps.items():
        if not r > 0:
            raise ValueError(f"link {l} has no positive rate ({r})")
    n = len(vals)
    median = vals[n // 2] if n % 2 else 0.5 * (vals[n // 2 - 1] + vals[n // 2])
    out = {}
    for l, r in sorted(rates_gbps.items()):
        out[l] = scale if r >= (1.0 - tolerance) * median else max(1, int(round(scale * median / r)))
    return out


def _link_name(link: Tuple[int, int]) -> str:
    a, b = link
    if b == LANE_OUT:
        return f"{a}->host"
    if a == LANE_IN:
        return f"host->{b}"
    if lane_pair_dst(b) is not None:
        return f"{a}->host->{lane_pair_dst(b)}"
    return f"{a}->{b}"


def choose_route(world: int, transfers: Sequence[Transfer], relay: bool = True,
                 rates_gbps: Optional[Dict[Tuple[int, int], float]] = None,
                 tolerance: float = 0.15, message_us: float = 0.0,
                 units: Sequence[int] = (64, 16), lane_chunk_bytes: int = 0) -> Tuple["RoutePlan", dict]:
    """The route plan for measured link rates: the uniform plan, the plan weighed by
    ``link_costs_from_rates`` (when some link is slower than the tolerance) and the direct-only
    plan, each at every ``units`` count (fewer parts per row, fewer messages), priced with
    ``RoutePlan.predicted_ms`` at the measured rates and per-message cost; the fastest is kept
    (ties to the earlier candidate, in that order: uniform at 64 parts first). When
    ``rates_gbps`` also holds the host lane's pseudo-links (``linkprobe.probe_lane``) every
    candidate is offered again with the lane (``+lane``, priced with the lane pipeline's fill of
    one ``lane_chunk_bytes`` chunk), after the lane-free ones. Deterministic: every rank holding
    the same measurements keeps the same plan. Without rates, the uniform plan at ``units[0]``
    without the lane. Returns (plan, report)."""
    uniform = RoutePlan(world, transfers, relay=relay, units=units[0])
    if not rates_gbps:
        return uniform, {"chosen": "uniform", "candidates": {}}
    lane_ok = any(is_lane_link(l) for l in rates_gbps)
    xgmi = {l: r for l, r in rates_gbps.items() if not is_lane_link(l)}
    pairs = priced_pairs(rates_gbps)  # cross-socket lane pairs with a rate of their own
    costs = link_costs_from_rates(rates_gbps, tolerance=tolerance)
    msg = max(0.0, float(message_us or 0.0))
    cands = []
    for lane in ([False, True] if lane_ok else [False]):
        sfx = "+lane" if lane else ""
        for u in units:
            base = uniform if (u == units[0] and not lane) else \
                RoutePlan(world, transfers, relay=relay, units=u, lane=lane, lane_pairs=pairs)
            tag = ("" if u == units[0] else f"/{u}") + sfx
            cands.append(("uniform" + tag, base))
            if costs and len(set(costs.values())) > 1:
                cands.append(("measured" + tag, RoutePlan(world, transfers, relay=relay, link_cost=costs, units=u,
                                                         lane=lane, lane_pairs=pairs)))
            if base.relay:
                cands.append(("direct" + tag, RoutePlan(world, transfers, relay=False, units=u, lane=lane,
                                                        lane_pairs=pairs)))
            if msg <= 0:
                break  # without a per-message cost, fewer parts can only lengthen the critical path
    scored = [(p.predicted_ms(rates_gbps, message_us=msg, lane_chunk_bytes=lane_chunk_bytes), i, name, p)
              for i, (name, p) in enumerate(cands)]
    best = min(scored, key=lambda x: (round(x[0], 9), x[1]))
    return best[3], {"chosen": best[2], "candidates": {name: round(t, 4) for t, _, name, _ in scored},
                     "message_us": round(msg, 2), "lane_offered": lane_ok,
                     "lane_pairs_priced": sorted([a, b] for a, b in pairs),
                     "slow_links": sorted(_link_name(l) for l, c in costs.items() if c != 16 and l in xgmi)}


def ring_transfers(dev_world: int, L: int, hl: int, hr: int, P: int, slice_world: int = 1,
                   slice_bounds: Optional[Sequence[int]] = None) -> List[Transfer]:
    """Global transfer list of a ring-window population in contiguous device blocks.

    Device block d (of ``dev_world``) sends its last ``hl`` rows to block d + 1's left halo and its
    first ``hr`` rows to block d - 1's right halo. With ``slice_world`` > 1 (hybrid partition)
    each block is held by ``slice_world`` ranks, rank = d * slice_world + p, each holding element
    slice p of every bucket (``slice_bounds``), and transfers stay within a slice. Element ranges
    are in the rank's own buffer coordinates: [0, slice length) of its slice, [0, P) without one.

    Stages: the left-halo row nearest the block (device first - 1, read by all hl left boundary
    devices) travels in stage 0, the farthest (device first - hl, read only by device 0) in stage
    hl - 1; likewise on the right."""
    if dev_world < 2:
        return []
    out: List[Transfer] = []
    for d in range(dev_world):
        left, right = (d - 1) % dev_world, (d + 1) % dev_world
        for p in range(slice_world):
            a, b = (slice_bounds[p], slice_bounds[p + 1]) if slice_bounds is not None else (0, P)
            me = d * slice_world + p
            for q in range(hl):
                out.append(Transfer(hl - 1 - q, left * slice_world + p, me, ("models", L - hl + q),
                                    ("left", q), 0, b - a))
            for q in range(hr):
                out.append(Transfer(q, right * slice_world + p, me, ("models", q), ("right", q), 0, b - a))
    out.sort(key=lambda t: (t.stage, t.dst, t.src, str(t.dst_key)))
    return out
