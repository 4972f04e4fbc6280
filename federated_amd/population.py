"""Sharded simulated-device population: one consensus round for all devices of a shard.

The reference simulates D devices as D OS processes on one host, each mixing its model with
its neighbours' models every round (TF1 ``FL_CFA_CNN_tf2.py:317-319``, TF2
``federated_learning_keras_consensus_FL_threads_CIFAR100.py:674-681``). Here the population is
device-resident: shard ``r`` of ``world`` owns devices ``[r*L, (r+1)*L)`` as one stacked
``[L, P]`` fp32 tensor in HBM (288 GB per MI355X holds thousands of 25M-parameter models).

Topology: a wrap-around ring window of ``h_left`` neighbours below and ``h_right`` above each
device (K = h_left + h_right): the symmetric form (h, h) is the wrap-around k-regular window
of ``get_connectivity`` (TF1 ``cfa.py:14-32``); (1, 0) is the TF2 v4 / FL_radar ring rule for
N < 2 (in-neighbour ii-1, ``consensus_v4.py:133-137``). Neighbour order is ascending device
offset (g-h_left, ..., g-1, g+1, ..., g+h_right), the order the reference's window lists them.
The mixing rule is the TF2 policy eps = 1/(K+1) applied sequentially (``consensus_v3.py:145,
153-155``).

A round = (1) halo exchange: the h_right first / h_left last buckets of each shard go to the
previous / next shard (one RCCL message per bucket, over xGMI), overlapped with (2) the mixes of
the interior devices, which need no remote bucket, then (3) the mixes of the boundary devices.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch


class RingShardPlan:
    """Index bookkeeping for one shard (pure host logic; testable on CPU)."""

    def __init__(self, rank: int, world: int, devices_per_shard: int, half_window: int,
                 right_window: Optional[int] = None):
        hl = half_window
        hr = half_window if right_window is None else right_window
        if devices_per_shard < 1 or hl < 0 or hr < 0:
            raise ValueError("need >= 1 device per shard and non-negative windows")
        if world > 1 and devices_per_shard < max(hl, hr):
            raise ValueError("a shard must hold at least as many devices as each window side")
        if hl + hr >= devices_per_shard * world:
            raise ValueError("ring window wider than the population")
        self.rank, self.world = rank, world
        self.L, self.hl, self.hr = devices_per_shard, hl, hr
        self.h = max(hl, hr)
        self.D = devices_per_shard * world
        self.first = rank * devices_per_shard
        self.left = (rank - 1) % world
        self.right = (rank + 1) % world

    @property
    def K(self) -> int:
        return self.hl + self.hr

    def neighbours(self, g: int) -> List[int]:
        """Global neighbour ids of global device g, in mixing order."""
        D = self.D
        return [(g + o) % D for o in list(range(-self.hl, 0)) + list(range(1, self.hr + 1))]

    def locate(self, g: int) -> Tuple[str, int]:
        """Where global device g's bucket lives on this shard: ('local', row), ('left', row) or
        ('right', row) of the halo buffers."""
        rel = (g - self.first) % self.D
        if rel < self.L:
            return "local", rel
        if self.world == 1:
            raise KeyError(g)
        if self.hl and rel >= self.D - self.hl:  # just below our first device: left halo
            return "left", rel - (self.D - self.hl)
        if self.hr and rel < self.L + self.hr:   # just above our last device: right halo
            return "right", rel - self.L
        raise KeyError(f"device {g} is not reachable from shard {self.rank}")

    def needs_halo(self, i: int) -> bool:
        """Does local device i (0-based in the shard) read a remote bucket?"""
        if self.world == 1:
            return False
        return i < self.hl or i >= self.L - self.hr

    def interior(self) -> List[int]:
        return [i for i in range(self.L) if not self.needs_halo(i)]

    def boundary(self) -> List[int]:
        return [i for i in range(self.L) if self.needs_halo(i)]

    def halo_transfers(self):
        """(sends, recvs): sends = [(local row, peer)], recvs = [((halo name, row), peer)], one
        bucket per message. The order makes the k-th send to a peer match that peer's k-th
        receive even when world == 2 (left == right peer): first the buckets that become the
        right neighbour's LEFT halo (our last hl rows, ascending), then those that become the
        left neighbour's RIGHT halo (our first hr rows); receives left halo rows, then right."""
        if self.world == 1:
            return [], []
        sends = [(r, self.right) for r in range(self.L - self.hl, self.L)]
        sends += [(r, self.left) for r in range(self.hr)]
        recvs = [(("left", r), self.left) for r in range(self.hl)]
        recvs += [(("right", r), self.right) for r in range(self.hr)]
        return sends, recvs


def row_checksum(t: torch.Tensor) -> int:
    """Exact, order-independent checksum of an fp32 row: the sum of its 32-bit patterns in int64
    (any single changed element changes it; computed where the row lives)."""
    return int(t.contiguous().view(torch.int32).to(torch.int64).sum().item())


def _overlaps(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Do the byte ranges of two tensors intersect (same device)?"""
    if a.device != b.device or a.numel() == 0 or b.numel() == 0:
        return False
    a0, b0 = a.data_ptr(), b.data_ptr()
    return a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()


def scattered_order(devices: List[int], K: int) -> List[int]:
    """``devices`` reordered so that consecutive mixes share no ring-window rows: a stride of
    3 (K + 1) through the list (every mix's K + 1 input rows are disjoint from the previous two
    mixes' rows when the list is long enough; shorter lists fall back to the largest stride that
    keeps one mix apart). Used to time a round whose rows the Infinity Cache cannot re-serve
    between consecutive mixes (bench.py's ``cache_reuse`` legs); the round's result is the same."""
    n = len(devices)
    s = 3 * (K + 1)
    while s > 1 and n < 2 * s:
        s //= 2
    if s <= 1:
        return list(devices)
    return [devices[i] for r in range(s) for i in range(r, n, s)]


def slice_bounds(P: int, parts: int, align: int = 64) -> List[int]:
    """Element slice bounds of a P-element bucket split in ``parts`` contiguous, ``align``-aligned
    slices (the last takes the remainder): slice p is [b[p], b[p + 1])."""
    units = -(-P // align)
    base, extra = divmod(units, parts)
    b = [0]
    for p in range(parts):
        b.append(min(P, b[-1] + (base + (1 if p < extra else 0)) * align))
    b[-1] = P
    return b


PARTITIONS = ("devices", "params", "hybrid")


def partition_shape(partition: str, world: int, devices: int, dev_groups: Optional[int] = None
                    ) -> Tuple[int, int]:
    """(device groups Gd, parameter slices Gp) with Gd * Gp = world.

    - ``devices``: contiguous device blocks, one per rank (Gd = world), SURVEY §8 e "Partitioning";
      a round exchanges the ring halo between neighbouring blocks.
    - ``params``: every rank holds all devices but only a 1/world element slice of every bucket
      (Gp = world), SURVEY §8 e "(1) within one bucket: elements are independent"; no exchange.
    - ``hybrid``: ``dev_groups`` device blocks, each split over world / dev_groups element
      slices; the halo moves between the ranks holding the same slice of neighbouring blocks."""
    if partition == "devices":
        gd, gp = world, 1
    elif partition == "params":
        gd, gp = 1, world
    elif partition == "hybrid":
        if not dev_groups or world % dev_groups:
            raise ValueError("hybrid partition needs dev_groups dividing the world size")
        gd, gp = dev_groups, world // dev_groups
    else:
        raise ValueError(f"unknown partition {partition!r} (one of {PARTITIONS})")
    if devices % gd:
        raise ValueError(f"{devices} devices do not split into {gd} equal blocks")
    return gd, gp


class RingPopulationShard:
    """Device-resident buckets of one shard plus its halo buffers, and the round itself."""

    def __init__(self, plan: RingShardPlan, P: int, device, transport=None, engine=None,
                 dtype=torch.float32, window_batch: int = 0, route=None, rank: Optional[int] = None,
                 stacks: Optional[Tuple[torch.Tensor, torch.Tensor]] = None, carve: bool = False):
        """``window_batch`` = B > 0 mixes B consecutive devices per ``cfa_mix_window_f32`` pass,
        loading each row of their shared window once (identical results); 0 = one streaming
        mix per device.

        ``route`` (a ``halo.RoutePlan`` over the global ranks, e.g. from ``make_ring_shard``)
        replaces the single grouped exchange: the halo travels in stages over direct and relayed
        paths, and each boundary device mixes as soon as the stages it reads have landed.
        ``rank`` is this shard's global rank in that plan (default ``plan.rank``).

        ``stacks`` = (models, mixed): caller-allocated ``[L, P]`` stacks (e.g. placement-calibrated,
        ``federated_amd.placement``) instead of fresh ones. ``carve`` (only for stacks from
        ``placement.calibrated_stacks``, which heads an allocation of 16 GiB or more with the
        models stack; ``make_ring_shard`` sets it) cuts the halo rows and the relay slots from the
        spare part of the models stack's allocation, so they share its placement. A carve that
        would overlap the ``mixed`` stack (stacks cut from one caller allocation) is refused and
        the halo is allocated on its own, as it is without ``carve``."""
        if window_batch and not (1 <= window_batch <= 8 and plan.hl <= 4 and plan.hr <= 4):
            raise ValueError("window_batch must be 1..8 with at most 4 neighbours per side")
        self.window_batch = int(window_batch)
        self.plan, self.P = plan, int(P)
        self.device = torch.device(device)
        if stacks is not None:
            for t in stacks:
                same_dev = t.device.type == self.device.type and (self.device.index is None
                                                                   or t.device.index == self.device.index)
                if tuple(t.shape) != (plan.L, self.P) or t.dtype != dtype or not same_dev:
                    raise ValueError(f"stacks must be [{plan.L}, {self.P}] {dtype} on {self.device}")
            self.models, self.mixed = stacks
        else:
            self.models = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
            self.mixed = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
        self.rank = plan.rank if rank is None else int(rank)
        self.route = route  # as given (None: the direct plan below)
        if route is None and plan.world > 1:
            route = self._direct_route()
        slot = route.slot_elems(self.rank) if route is not None else 0
        carved = None
        if stacks is not None and carve and plan.world > 1:
            from .placement import spare_view
            carved = spare_view(self.models, [(plan.hl, self.P), (plan.hr, self.P), (2, max(slot, 1))])
            if carved is not None and any(_overlaps(v, self.mixed) for v in carved):
                carved = None
        if carved is not None:
            self.halo = {"left": carved[0], "right": carved[1]}
            self._relay_buf = carved[2]
        else:
            self.halo = {
                "left": torch.empty((plan.hl, self.P), dtype=dtype, device=self.device),
                "right": torch.empty((plan.hr, self.P), dtype=dtype, device=self.device),
            }
            self._relay_buf = None
        self.carved = carved is not None
        self.transport = transport
        self.engine = engine
        self.alphas = [1.0 / (plan.K + 1)] * plan.K
        self._route_plan = route
        self._routed = None
        self.lane = None  # hostlane.HostLane, when the route puts pieces on the host lane (open_lane)
        # order of the interior mixes within a round (None: ascending device id, the ring order);
        # the mixes write a separate stack, so any order gives the same round
        self.mix_order: Optional[List[int]] = None
        self._launch = {}
        # stage after which each boundary device can mix (the latest stage of the halo rows it reads)
        self._ready = {}
        if route is not None:
            stage_of = {}
            for t in route.transfers:
                if t.dst == self.rank:
                    stage_of[t.dst_key] = t.stage
            for i in self.plan.boundary():
                g = plan.first + i
                st = [stage_of[self.plan.locate(j)] for j in plan.neighbours(g) if self.plan.locate(j)[0] != "local"]
                self._ready[i] = max(st) if st else -1

    def _direct_route(self):
        """One-stage, direct-only plan: the grouped exchange of round 1 (every halo bucket one
        message on its direct link)."""
        from .halo import RoutePlan, ring_transfers
        p = self.plan
        tr = [t for t in ring_transfers(p.world, p.L, p.hl, p.hr, self.P)]
        tr = [type(t)(0, t.src, t.dst, t.src_key, t.dst_key, t.lo, t.hi) for t in tr]
        return RoutePlan(p.world, tr, relay=False)

    def buffer(self, key) -> torch.Tensor:
        """Row tensor of a route key: ("models", row), ("left", row) or ("right", row)."""
        name, row = key
        return self.models[row] if name == "models" else self.halo[name][row]

    def bucket(self, g: int) -> torch.Tensor:
        where, row = self.plan.locate(g)
        return self.models[row] if where == "local" else self.halo[where][row]

    def sources(self, i: int) -> List[torch.Tensor]:
        g = self.plan.first + i
        return [self.bucket(j) for j in self.plan.neighbours(g)]

    def routed(self):
        """The RoutedExchange of this shard (built on first use: it allocates relay staging)."""
        if self._routed is None and self._route_plan is not None:
            from .halo import RoutedExchange
            self._routed = RoutedExchange(self._route_plan, self.rank, self.buffer, self.transport,
                                          self.device, self.models.dtype, relay=self._relay_buf, lane=self.lane)
        return self._routed

    def open_lane(self, token: str, agree, **kw) -> None:
        """Open the host lane of the route (collective: every rank of the plan calls it with the
        same ``token``; ``agree(ok)`` is the control plane's all-ranks AND; ``kw`` goes to
        ``HostLane``, e.g. ``numa_nodes``). A no-op for a route without lane pieces anywhere."""
        route = self._route_plan
        if route is None or not route.lane:
            return
        from .hostlane import HostLane
        sends, recvs = route.lane_ops(self.rank)
        self.lane = HostLane.open(self.rank, sends, recvs, self.buffer, self.device, token, agree, **kw)
        self._routed = None

    def exchange(self, stream=None) -> None:
        """The whole halo exchange, issued on ``stream`` (synchronous for host transports; the host
        lane's part is finished on the host before this returns)."""
        r = self.routed()
        if r is not None:
            r.run(stream)
            r.finish_lane()

    def close(self) -> None:
        """Release the shard's host lane (unpin and unmap its segments); the stacks go with the
        object. Every path that drops a shard with a lane calls this."""
        if self.lane is not None:
            self.lane.close()
            self.lane = None
            self._routed = None

    def mix_device(self, i: int, stream=None) -> None:
        fn = self._launch.get(i)
        if fn is None and self.engine is not None:
            fn = self._launch[i] = self.engine.prepare_mix_seq(self.mixed[i], self.models[i], self.sources(i),
                                                              self.alphas)
        fn(stream)

    def interior_order(self) -> List[int]:
        """The interior devices in the order a round mixes them."""
        return list(self.mix_order) if self.mix_order is not None else self.plan.interior()

    def window_passes(self, devices: List[int]) -> List[List[int]]:
        """Runs of consecutive local devices, cut into passes of at most window_batch."""
        passes, run = [], []
        for i in devices:
            if run and (i != run[-1] + 1 or len(run) == self.window_batch):
                passes.append(run)
                run = []
            run.append(i)
        if run:
            passes.append(run)
        return passes

    def mix_window(self, devs: List[int], stream=None) -> None:
        """One cfa_mix_window_f32 pass over consecutive local devices devs."""
        p = self.plan
        g0 = p.first + devs[0]
        rows = [self.bucket((g0 + o) % p.D) for o in range(-p.hl, len(devs) + p.hr)]
        self.engine.mix_window([self.mixed[i] for i in devs], rows, [self.alphas] * len(devs), p.hl, p.hr, stream)

    def _mix_set(self, devices: List[int], stream, timer=None, between=None) -> None:
        """Mix ``devices`` on ``stream``; ``between()`` (optional) after each launch (the host
        lane's non-blocking pump, so an H2D whose chunk has arrived is enqueued at once)."""
        if self.window_batch:
            for run in self.window_passes(devices):
                if timer:
                    timer(run[0], True)
                self.mix_window(run, stream)
                if timer:
                    timer(run[-1], False)
                if between:
                    between()
            return
        for i in devices:
            if timer:
                timer(i, True)
            self.mix_device(i, stream)
            if timer:
                timer(i, False)
            if between:
                between()

    def halo_check(self, gather, slice_lo: int = 0) -> Tuple[int, int]:
        """After an exchange: every halo row against the row its owner holds, by ``row_checksum``.
        ``gather(obj)`` returns every rank's ``obj`` (torch.distributed.all_gather_object); each
        rank contributes the rows other shards read (its first ``hr`` and last ``hl``), keyed by
        (global device, ``slice_lo``) so the slices of a hybrid partition stay apart. Collective.
        Returns (halo rows checked, rows that differ) on this rank."""
        p = self.plan
        own = {(p.first + i, int(slice_lo)): row_checksum(self.models[i])
               for i in range(p.L) if p.world > 1 and (i < p.hr or i >= p.L - p.hl)}
        table = {}
        for part in gather(own):
            table.update(part or {})
        if p.world == 1:
            return 0, 0
        rows = [((p.first - p.hl + q) % p.D, self.halo["left"][q]) for q in range(p.hl)]
        rows += [((p.first + p.L + q) % p.D, self.halo["right"][q]) for q in range(p.hr)]
        bad = sum(row_checksum(r) != table.get((g, int(slice_lo))) for g, r in rows)
        return len(rows), int(bad)

    @property
    def route_plan(self):
        """The halo.RoutePlan this shard exchanges with (None at world 1)."""
        return self._route_plan

    def compute_round(self, stream=None, timer=None) -> None:
        """Every device's mix and nothing else (the halo rows hold what the last exchange
        delivered): the compute-only round of the bench's N > 1 decomposition. ``timer`` as in
        ``round``, around every mix."""
        cs = stream or torch.cuda.current_stream(self.device)
        self._mix_set(self.interior_order() + self.plan.boundary(), cs, timer)

    def boundary_schedule(self) -> List[Tuple[int, int]]:
        """[(exchange group after which they can mix, number of boundary devices)], in the order a
        round mixes them (host logic; ``predict_round_ms``'s input)."""
        route = self._route_plan
        if route is None:
            return []
        return [(route.done_group(stage), len(devs)) for stage, devs in self.stage_sets()]

    def stage_sets(self) -> List[Tuple[int, List[int]]]:
        """[(stage, boundary devices that can mix once that stage has landed)], stage order."""
        by = {}
        for i, s in self._ready.items():
            by.setdefault(s, []).append(i)
        return [(s, sorted(by[s])) for s in sorted(by)]

    def round(self, compute_stream: Optional[torch.cuda.Stream] = None,
              comm_stream: Optional[torch.cuda.Stream] = None, timer=None) -> None:
        """One consensus round: the halo exchange on ``comm_stream`` overlapped with the interior
        mixes on ``compute_stream``; each boundary device mixes once the stages it reads have
        landed. ``timer`` (optional) is called as timer(i, start) around each interior mix."""
        cs = compute_stream or torch.cuda.current_stream(self.device)
        routed = self.routed() if self.plan.world > 1 else None
        if routed is None:
            self._mix_set(self.interior_order(), cs, timer)
            self._mix_set(self.plan.boundary(), cs)
            return
        ms = comm_stream or cs
        on_gpu = ms.device.type == "cuda" if hasattr(ms, "device") else True
        # a transport that blocks the host (gloo's host staging) would hold the interior mixes back
        # until the whole exchange is done: then they are enqueued first, and the exchange waits only
        # for the models being final (an event before them), not for the mixes
        early = bool(getattr(self.transport, "host_staged", False)) and on_gpu and ms is not cs
        if early:
            ready = torch.cuda.Event()
            ready.record(cs)
            ms.wait_event(ready)
        else:
            ms.wait_stream(cs)  # models are ready (e.g. written by SGD) before they leave
        sets = self.stage_sets()
        events = {}

        def landed(stage):
            if on_gpu and ms is not cs:
                ev = torch.cuda.Event()
                ev.record(ms)
                events[stage] = ev

        pump = routed.lane.pump if routed.lane is not None else None

        def interior():
            self._mix_set(self.interior_order(), cs, timer, pump)
        routed.run(ms, landed, before_groups=interior if early else None)
        if not early:
            interior()
        for stage, devs in sets:
            ev = events.get(stage)
            if ev is not None:
                cs.wait_event(ev)
            elif ms is not cs:
                cs.wait_stream(ms)
            lev = routed.lane_event(stage) if routed.lane is not None else None
            if lev is not None:
                cs.wait_event(lev)  # a hostlane.LaneGate: pumps the lane on the host, then waits
            self._mix_set(devs, cs, between=pump)
        if ms is not cs:
            cs.wait_stream(ms)  # the next round's exchange must not overwrite a halo still read
        if routed.lane is not None:
            if on_gpu:
                routed.lane.wait_streams(cs)  # nor the lane's; and the rows have left before they change
            else:
                routed.lane.finish()

    @property
    def bytes_per_round(self) -> int:
        """Algorithmic HBM bytes of the mixes: (K + 2) * P * 4 per device."""
        return self.plan.L * (self.plan.K + 2) * self.P * self.models.element_size()


def predict_round_ms(group_ms: List[float], schedule: List[Tuple[int, int]], n_interior: int, t_mix_ms: float,
                     delta: float, lane_ready_ms: Optional[List[Optional[float]]] = None,
                     lane_end_ms: float = 0.0) -> float:
    """Length of one overlapped round from its measured parts (the bench's N > 1 decomposition):
    the exchange groups run back to back from t = 0 on the comm stream (``group_ms``, measured
    with no mixes); the compute stream mixes the ``n_interior`` interior devices from t = 0, then
    each boundary set of ``schedule`` [(group, devices)] once its group has landed. A mix takes
    ``t_mix_ms`` (measured with no exchange) stretched by (1 + ``delta``) while the exchange is
    still running (RCCL's copy kernels share the CUs and HBM; ``delta`` measured from the
    headline's own interior mixes), ``t_mix_ms`` after it. With the host lane,
    ``lane_ready_ms[i]`` (per schedule entry, None = nothing of it on the lane) is when the lane's
    pieces of that boundary set have landed (measured from the exchange's start) and
    ``lane_end_ms`` when the lane's last copy ends: a set waits for both paths, and the exchange
    lasts until both are done."""
    ends, t = [], 0.0
    for g in group_ms:
        t += g
        ends.append(t)
    t_x = max(ends[-1] if ends else 0.0, lane_end_ms)

    def mixes(n, t):
        for _ in range(n):
            t += t_mix_ms * (1.0 + delta) if t < t_x else t_mix_ms
        return t

    t = mixes(n_interior, 0.0)
    for i, (g, n) in enumerate(schedule):
        if ends:
            t = max(t, ends[min(g, len(ends) - 1)])
        if lane_ready_ms and i < len(lane_ready_ms) and lane_ready_ms[i] is not None:
            t = max(t, lane_ready_ms[i])
        t = mixes(n, t)
    return max(t, t_x)


def make_ring_shard(rank: int, world: int, devices: int, hl: int, hr: int, P: int, device,
                    transport=None, engine=None, partition: str = "devices",
                    dev_groups: Optional[int] = None, relay: bool = True, staged: bool = True,
                    window_batch: int = 0, dtype=torch.float32, placement_candidates: int = 0,
                    placement_release: bool = False, link_rates=None, message_us: float = 0.0,
                    lane_token: Optional[str] = None, lane_agree=None, lane_chunk_elems: Optional[int] = None,
                    lane_numa_nodes=None):
    """The shard of global rank ``rank`` for a fixed population of ``devices`` ring devices
    (strong scaling: the population does not grow with ``world``).

    Returns (shard, info): ``shard.P`` is this rank's slice length and ``info`` holds the
    partition, its (Gd, Gp) shape, this rank's element slice [lo, hi) of every bucket and the
    route summary. ``relay`` spreads the halo over relayed xGMI paths; ``staged`` sends it row by
    row so boundary devices mix as their rows land (both only matter when Gd > 1).
    ``placement_candidates`` > 1 allocates the shard's stacks placement-calibrated
    (``placement.calibrated_stacks``: the fastest of that many allocations each, timed with the
    shard's own mix; ``info["placement"]`` holds the probe). ``link_rates``: measured per-link rates
    (GB/s, ``linkprobe.probe_links``): the route is then ``halo.choose_route``'s pick among the
    uniform, the rate-weighted and the direct plan, at 64 and (with a per-message cost
    ``message_us`` > 0) 16 parts per row (``info["route_choice"]``); None = every link alike.
    When ``link_rates`` also holds the host lane's pseudo-links (``linkprobe.probe_lane``) the lane
    is offered to the route too; if the chosen route uses it the shard's lane is opened here
    (collective: every rank passes the same ``lane_token`` and ``lane_agree``, the control plane's
    all-ranks AND; ``lane_numa_nodes[r]``: the NUMA node of rank r's GPU, where the segments rank
    r receives are placed)."""
    from .halo import choose_route, ring_transfers
    gd, gp = partition_shape(partition, world, devices, dev_groups)
    d, p = divmod(rank, gp)
    bounds = slice_bounds(P, gp)
    L = devices // gd
    plan = RingShardPlan(d, gd, L, hl, hr)
    route, route_choice = None, None
    if gd > 1:
        tr = ring_transfers(gd, L, hl, hr, P, slice_world=gp, slice_bounds=bounds)
        if not staged:
            tr = [type(t)(0, t.src, t.dst, t.src_key, t.dst_key, t.lo, t.hi) for t in tr]
        from .hostlane import DEFAULT_CHUNK_ELEMS, first_chunk_elems
        chunk = int(lane_chunk_elems or DEFAULT_CHUNK_ELEMS)
        route, route_choice = choose_route(world, tr, relay=relay, rates_gbps=link_rates, message_us=message_us,
                                           lane_chunk_bytes=first_chunk_elems(chunk) * 4)
        if route.lane and (lane_token is None or lane_agree is None):
            raise ValueError("the chosen route uses the host lane: make_ring_shard needs lane_token and lane_agree")
    Pr = bounds[p + 1] - bounds[p]
    stacks, placement = None, None
    if placement_candidates > 1 and engine is not None and torch.device(device).type == "cuda":
        from .placement import calibrated_stacks
        models, mixed, placement = calibrated_stacks(L, Pr, device, engine, hl, hr, placement_candidates,
                                                     dtype=dtype, release=placement_release)
        stacks = (models, mixed)
    shard = RingPopulationShard(plan, Pr, device, transport, engine, dtype, window_batch, route=route, rank=rank,
                                stacks=stacks, carve=stacks is not None)
    if route is not None and route.lane:
        shard.open_lane(lane_token, lane_agree, chunk_elems=chunk, numa_nodes=lane_numa_nodes)
    info = {"partition": partition, "device_groups": gd, "param_slices": gp,
            "slice": [bounds[p], bounds[p + 1]], "first_device": plan.first, "devices_per_rank": L,
            "placement": placement, "halo_carved": shard.carved}
    if route is not None:
        info["route"] = route.summary()
        info["route_digest"] = route.digest()
        info["route_choice"] = route_choice
        if shard.lane is not None:
            info["lane"] = shard.lane.summary()
    return shard, info
