"""Sharded simulated-device population on an ARBITRARY topology (SURVEY §8 e, "random / vGraph /
np.random.choice neighbours: grouped send/recv by CSR").

``population.py`` shards the ring window, whose halo is a fixed band. Here the neighbour lists
come from the topology service (``topology.py``: k-regular ``cfa.py:14-32``, ``consensus_v3.py:44-70``,
ring ``consensus_v4.py:111-141``, vGraph rows with the ``random.choices`` draw of
``cfa_ongraphs.py:33-52``), computed identically on every rank from the same seeds. Shard ``r`` of
``world`` owns the contiguous device block ``[first, first + L)``:

- its halo is the sorted set of remote devices its devices read;
- it sends each peer the peer's needed devices of its own block in ascending device id, so the
  k-th message to a peer pairs with that peer's k-th receive from us (one RCCL message per
  bucket, grouped, no handshake);
- a round is: exchange on the comm stream, overlapped with the interior devices (no remote
  neighbour), then the boundary devices once the halo has landed.

Mixing rule: the sequential CFA rule with per-device alphas from an eps policy
(``topology.alphas_*``), on fp32 buckets. Small buckets mix in one ``cfa_mix_population_f32``
launch per device set. Large ones use one streaming ``mix_vec_kernel`` launch per device, which
was measured faster at P = 25M.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import topology as T

POPULATION_LAUNCH_MAX_P = 1 << 21  # at or below: one population launch per device set


def block_bounds(D: int, world: int) -> List[int]:
    """Contiguous blocks as even as possible: rank r owns [b[r], b[r+1])."""
    base, extra = divmod(D, world)
    b = [0]
    for r in range(world):
        b.append(b[-1] + base + (1 if r < extra else 0))
    return b


class GraphShardPlan:
    def __init__(self, lists: Sequence[Sequence[int]], rank: int, world: int):
        self.lists = [[int(j) for j in nb] for nb in lists]
        self.D, self.rank, self.world = len(self.lists), int(rank), int(world)
        if not 0 <= self.rank < self.world or self.world > self.D:
            raise ValueError(f"bad rank/world {rank}/{world} for {self.D} devices")
        self.bounds = block_bounds(self.D, self.world)
        self.first, self.L = self.bounds[self.rank], self.bounds[self.rank + 1] - self.bounds[self.rank]
        for d, nb in enumerate(self.lists):
            if any(not 0 <= j < self.D for j in nb):
                raise ValueError(f"device {d}: neighbour out of range")
        own = range(self.first, self.first + self.L)
        self.halo_devices = sorted({j for d in own for j in self.lists[d] if self.owner(j) != self.rank})
        self._halo_row = {g: h for h, g in enumerate(self.halo_devices)}

    def owner(self, g: int) -> int:
        return int(np.searchsorted(self.bounds, g, side="right") - 1)

    def neighbours(self, g: int) -> List[int]:
        return self.lists[g]

    def locate(self, g: int) -> Tuple[str, int]:
        """('local', row) or ('halo', row) of global device g as seen by this shard."""
        if self.first <= g < self.first + self.L:
            return "local", g - self.first
        if g in self._halo_row:
            return "halo", self._halo_row[g]
        raise KeyError(f"device {g} is neither local to shard {self.rank} nor in its halo")

    def needs_halo(self, i: int) -> bool:
        return any(self.owner(j) != self.rank for j in self.lists[self.first + i])

    def interior(self) -> List[int]:
        return [i for i in range(self.L) if not self.needs_halo(i)]

    def boundary(self) -> List[int]:
        return [i for i in range(self.L) if self.needs_halo(i)]

    def halo_transfers(self):
        """(sends, recvs): sends = [(local row, peer)], recvs = [(halo row, peer)], one bucket per
        message; per peer pair both sides list the buckets in ascending device id."""
        sends, recvs = [], []
        for p in range(self.world):
            if p == self.rank:
                continue
            theirs = range(self.bounds[p], self.bounds[p + 1])
            need = sorted({j for d in theirs for j in self.lists[d] if self.owner(j) == self.rank})
            sends += [(g - self.first, p) for g in need]
        recvs = [(h, self.owner(g)) for h, g in enumerate(self.halo_devices)]
        return sends, recvs


class GraphPopulationShard:
    """Device-resident buckets of one shard, its halo buffers, CSR tables and the round."""

    def __init__(self, plan: GraphShardPlan, P: int, device, transport=None, engine=None,
                 policy: Callable = T.alphas_tf2, dtype=torch.float32, placement_candidates: int = 0):
        """``placement_candidates`` > 1: the models / mixed stacks are placement-calibrated
        (``placement.calibrated_stacks``, probed with ring-window mixes of the same shapes; the
        level is a property of the allocation, not of the topology) when the round runs
        per-device streaming mixes (P above POPULATION_LAUNCH_MAX_P); ``self.placement`` holds
        the probe."""
        self.plan, self.P = plan, int(P)
        self.device = torch.device(device)
        self.placement = None
        if (placement_candidates > 1 and engine is not None and self.device.type == "cuda"
                and self.P > POPULATION_LAUNCH_MAX_P):
            from .placement import calibrated_stacks
            h = min(4, max(1, (plan.L - 1) // 2))
            self.models, self.mixed, self.placement = calibrated_stacks(
                plan.L, self.P, self.device, engine, h, h, placement_candidates, dtype=dtype)
        else:
            self.models = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
            self.mixed = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
        carved = None
        if self.placement is not None and plan.halo_devices:
            from .placement import spare_view  # halo rows on the calibrated models allocation
            carved = spare_view(self.models, [(len(plan.halo_devices), self.P)])
        self.halo = carved[0] if carved is not None else torch.empty((len(plan.halo_devices), self.P), dtype=dtype,
                                                                      device=self.device)
        self.transport, self.engine = transport, engine
        self.alphas = [list(policy(plan.lists[plan.first + i], plan.first + i, plan.D)) for i in range(plan.L)]
        self._tables = {}
        if engine is not None and self.P <= POPULATION_LAUNCH_MAX_P:
            for name, subset in (("interior", plan.interior()), ("boundary", plan.boundary())):
                self._tables[name] = self._build_tables(subset)

    def bucket(self, g: int) -> torch.Tensor:
        where, row = self.plan.locate(g)
        return self.models[row] if where == "local" else self.halo[row]

    def sources(self, i: int) -> List[torch.Tensor]:
        return [self.bucket(j) for j in self.plan.neighbours(self.plan.first + i)]

    def _build_tables(self, subset: Sequence[int]):
        """CSR over the source table [models rows..., halo rows...] for the devices in subset."""
        if not subset:
            return None
        L = self.plan.L
        src = [self.models[r].data_ptr() for r in range(L)] + [self.halo[h].data_ptr() for h in range(self.halo.shape[0])]
        ptr, idx, coef = [0], [], []
        for i in subset:
            idx.append(i)
            coef.append(1.0)
            for j, a in zip(self.plan.neighbours(self.plan.first + i), self.alphas[i]):
                where, row = self.plan.locate(j)
                idx.append(row if where == "local" else L + row)
                coef.append(float(a))
            ptr.append(len(idx))
        dev = self.device
        return (torch.tensor([self.mixed[i].data_ptr() for i in subset], dtype=torch.int64, device=dev),
                torch.tensor(src, dtype=torch.int64, device=dev),
                torch.tensor(ptr, dtype=torch.int32, device=dev),
                torch.tensor(idx, dtype=torch.int32, device=dev),
                torch.tensor(coef, dtype=torch.float32, device=dev), len(subset))

    def exchange(self, stream=None) -> None:
        sends, recvs = self.plan.halo_transfers()
        if not sends and not recvs:
            return
        self.transport.exchange([(self.models[r], p) for r, p in sends],
                                [(self.halo[h], p) for h, p in recvs], stream)

    def _mix(self, name: str, subset: Sequence[int], stream) -> None:
        tabs = self._tables.get(name)
        if tabs is not None:
            out_ptrs, src_ptrs, ptr, idx, coef, n = tabs
            self.engine.population(out_ptrs, src_ptrs, ptr, idx, coef, n, T.RULE_SEQUENTIAL, self.P, stream)
            return
        for i in subset:
            self.engine.mix_seq(self.mixed[i], self.models[i], self.sources(i), self.alphas[i], stream)

    def round(self, compute_stream: Optional[torch.cuda.Stream] = None,
              comm_stream: Optional[torch.cuda.Stream] = None) -> None:
        cs = compute_stream or torch.cuda.current_stream(self.device)
        if self.plan.world > 1:
            ms = comm_stream or cs
            ms.wait_stream(cs)
            self.exchange(ms)
        self._mix("interior", self.plan.interior(), cs)
        if self.plan.world > 1:
            cs.wait_stream(comm_stream or cs)
        self._mix("boundary", self.plan.boundary(), cs)

    @property
    def bytes_per_round(self) -> int:
        esz = self.models.element_size()
        return sum((len(self.plan.neighbours(self.plan.first + i)) + 2) * self.P * esz for i in range(self.plan.L))
