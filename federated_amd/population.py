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


class RingPopulationShard:
    """Device-resident buckets of one shard plus its halo buffers, and the round itself."""

    def __init__(self, plan: RingShardPlan, P: int, device, transport=None, engine=None,
                 dtype=torch.float32, window_batch: int = 0):
        """``window_batch`` = B > 0 mixes B consecutive devices per ``cfa_mix_window_f32`` pass,
        loading each row of their shared window once (identical results); 0 = one streaming
        mix per device."""
        if window_batch and not (1 <= window_batch <= 8 and plan.hl <= 4 and plan.hr <= 4):
            raise ValueError("window_batch must be 1..8 with at most 4 neighbours per side")
        self.window_batch = int(window_batch)
        self.plan, self.P = plan, int(P)
        self.device = torch.device(device)
        self.models = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
        self.mixed = torch.empty((plan.L, self.P), dtype=dtype, device=self.device)
        self.halo = {
            "left": torch.empty((plan.hl, self.P), dtype=dtype, device=self.device),
            "right": torch.empty((plan.hr, self.P), dtype=dtype, device=self.device),
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
        s = [(self.models[row], peer) for row, peer in sends]
        r = [(self.halo[name][row], peer) for (name, row), peer in recvs]
        self.transport.exchange(s, r, stream)

    def mix_device(self, i: int, stream=None) -> None:
        self.engine.mix_seq(self.mixed[i], self.models[i], self.sources(i), self.alphas, stream)

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

    def _mix_set(self, devices: List[int], stream, timer=None) -> None:
        if self.window_batch:
            for run in self.window_passes(devices):
                if timer:
                    timer(run[0], True)
                self.mix_window(run, stream)
                if timer:
                    timer(run[-1], False)
            return
        for i in devices:
            if timer:
                timer(i, True)
            self.mix_device(i, stream)
            if timer:
                timer(i, False)

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
        self._mix_set(self.plan.interior(), cs, timer)
        if self.plan.world > 1:
            cs.wait_stream(comm_stream or cs)
        self._mix_set(self.plan.boundary(), cs)

    @property
    def bytes_per_round(self) -> int:
        """Algorithmic HBM bytes of the mixes: (K + 2) * P * 4 per device."""
        return self.plan.L * (self.plan.K + 2) * self.P * self.models.element_size()
