"""Sharded simulated-device population: one consensus round for all devices of a shard.

The reference simulates D devices as D OS processes on one host, each mixing its model with
its neighbours' models every round (TF1 ``FL_CFA_CNN_tf2.py:317-319``, TF2
``federated_learning_keras_consensus_FL_threads_CIFAR100.py:674-681``). Here the population is
device-resident: shard ``r`` of ``world`` owns devices ``[r*L, (r+1)*L)`` as one stacked
``[L, P]`` fp32 tensor in HBM (288 GB per MI355X holds thousands of 25M-parameter models).

Topology: a ring window of ``h`` in-neighbours on each side (K = 2h neighbours), the
wrap-around form of the k-regular window ``get_connectivity`` (TF1 ``cfa.py:14-32``) that
TF2 ``consensus_v4.py:133-137`` uses for its ring. Neighbour order is ascending device offset
(g-h, ..., g-1, g+1, ..., g+h), the order the reference's window lists them. The mixing rule is
the TF2 policy eps = 1/(K+1) applied sequentially (``consensus_v3.py:145,153-155``).

A round = (1) halo exchange: the h first / h last buckets of each shard go to the previous /
next shard (one message per side, RCCL over xGMI), overlapped with (2) the mixes of the
interior devices, which need no remote bucket, then (3) the mixes of the 2h boundary devices.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch


class RingShardPlan:
    """Index bookkeeping for one shard (pure host logic; testable on CPU)."""

    def __init__(self, rank: int, world: int, devices_per_shard: int, half_window: int):
        if devices_per_shard < 1 or half_window < 0:
            raise ValueError("need >= 1 device per shard and a non-negative window")
        if world > 1 and devices_per_shard < half_window:
            raise ValueError("a shard must hold at least `half_window` devices")
        if 2 * half_window >= devices_per_shard * world:
            raise ValueError("ring window wider than the population")
        self.rank, self.world = rank, world
        self.L, self.h = devices_per_shard, half_window
        self.D = devices_per_shard * world
        self.first = rank * devices_per_shard
        self.left = (rank - 1) % world
        self.right = (rank + 1) % world

    @property
    def K(self) -> int:
        return 2 * self.h

    def neighbours(self, g: int) -> List[int]:
        """Global neighbour ids of global device g, in mixing order."""
        h, D = self.h, self.D
        return [(g + o) % D for o in list(range(-h, 0)) + list(range(1, h + 1))]

    def locate(self, g: int) -> Tuple[str, int]:
        """Where global device g's bucket lives on this shard: ('local', row), ('left', row) or
        ('right', row) of the halo buffers."""
        rel = (g - self.first) % self.D
        if rel < self.L:
            return "local", rel
        if self.world == 1:
            raise KeyError(g)
        if rel >= self.D - self.h:  # just below our first device: left halo
            return "left", rel - (self.D - self.h)
        if rel < self.L + self.h:   # just above our last device: right halo
            return "right", rel - self.L
        raise KeyError(f"device {g} is not reachable from shard {self.rank}")

    def needs_halo(self, i: int) -> bool:
        """Does local device i (0-based in the shard) read a remote bucket?"""
        if self.world == 1:
            return False
        return i < self.h or i >= self.L - self.h

    def interior(self) -> List[int]:
        return [i for i in range(self.L) if not self.needs_halo(i)]

    def boundary(self) -> List[int]:
        return [i for i in range(self.L) if self.needs_halo(i)]

    def halo_transfers(self):
        """(sends, recvs) as (row slice of the local stack or halo name, peer). Order is chosen
        so that with world == 2 (left == right peer) the k-th send to a peer matches that peer's
        k-th receive: first the message that becomes the right neighbour's LEFT halo, then the one
        that becomes the left neighbour's RIGHT halo; receives left halo first, then right."""
        if self.world == 1 or self.h == 0:
            return [], []
        sends = [(slice(self.L - self.h, self.L), self.right), (slice(0, self.h), self.left)]
        recvs = [("left", self.left), ("right", self.right)]
        return sends, recvs


class RingPopulationShard:
    """Device-resident buckets of one shard plus its halo buffers, and the round itself."""

    def __init__(self, plan: RingShardPlan, P: int, device, transport=None, engine=None,
                 dtype=torch.float32):
        self.plan, self.P = plan, int(P)
        self.device = torch.device(device)
        h = plan.h
        self.models = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
        self.mixed = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
        self.halo = {
            "left": torch.empty((h, self.P), dtype=dtype, device=self.device),
            "right": torch.empty((h, self.P), dtype=dtype, device=self.device),
        }
        self.transport = transport
        self.engine = engine
        self.alphas = [1.0 / (plan.K + 1)] * plan.K

    def bucket(self, g: int) -> torch.Tensor:
        where, row = self.plan.locate(g)
        return self.models[row] if where == "local" else self.halo[where][row]

    def sources(self, i: int) -> List[torch.Tensor]:
        g = self.plan.first + i
        return [self.bucket(j) for j in self.plan.neighbours(g)]

    def exchange(self, stream=None) -> None:
        sends, recvs = self.plan.halo_transfers()
        if not sends and not recvs:
            return
        s = [(self.models[sl].reshape(-1), peer) for sl, peer in sends]
        r = [(self.halo[name].reshape(-1), peer) for name, peer in recvs]
        self.transport.exchange(s, r, stream)

    def mix_device(self, i: int, stream=None) -> None:
        self.engine.mix_seq(self.mixed[i], self.models[i], self.sources(i), self.alphas, stream)

    def round(self, compute_stream: Optional[torch.cuda.Stream] = None,
              comm_stream: Optional[torch.cuda.Stream] = None, timer=None) -> None:
        """One consensus round: halo exchange on ``comm_stream`` overlapped with interior mixes on
        ``compute_stream``, then the boundary mixes once the halo has landed. ``timer`` (optional)
        is called as timer(i, start) around each interior mix to time the kernel."""
        cs = compute_stream or torch.cuda.current_stream(self.device)
        if self.plan.world > 1:
            ms = comm_stream or cs
            ms.wait_stream(cs)  # models are ready (e.g. written by SGD) before they leave
            self.exchange(ms)
        for i in self.plan.interior():
            if timer:
                timer(i, True)
            self.mix_device(i, cs)
            if timer:
                timer(i, False)
        if self.plan.world > 1:
            cs.wait_stream(comm_stream or cs)
        for i in self.plan.boundary():
            self.mix_device(i, cs)

    @property
    def bytes_per_round(self) -> int:
        """Algorithmic HBM bytes of the mixes: (K + 2) * P * 4 per device."""
        return self.plan.L * (self.plan.K + 2) * self.P * self.models.element_size()
