"""FedAvg / parameter-server aggregation of a device population sharded over the GPUs of a node.

The reference's parameter server folds the C models it received into the global model one at a
time (TF2 ``parameter_server_v2.py:159-161``, ``parameter_server.py:154``; MQTT
``PS_server.py:130-133``):

    p <- p + u * (x_k - p) / C        for k = 0 .. C-1, in device order

and, when a device reports ``training_end``, takes the transfer-learning branch instead
(``parameter_server_v2.py:150-157``): p <- p + u * (x_e - p) for the first such device e.

With the population sharded one block of devices per rank ("PS/FedAvg (f1) ...
pre-scale on each rank, then ncclAllReduce(sum), or ncclReduce to the owner"), the fold is
evaluated in its closed form, which is linear in the models:

    p' = c_p * p + sum_k c_k * x_k,   a = u / C,   c_p = (1 - a)^C,   c_k = a * (1 - a)^(C-1-k)

(coefficients in fp64, rounded once to fp32). Each rank pre-scales and sums its own devices'
models in ONE streaming launch (``cfa_mix_f32``, the linear rule; rank 0 also folds in c_p * p),
then one RCCL sum all-reduce (``cfa_allreduce_sum_f32``) leaves p' on every rank, which is where
the next round's devices start from (the PS publishes p' to every device). ``reduce_to=r`` uses
``cfa_reduce_sum_f32`` instead, for a PS that lives on one rank.

Parity: the closed form and the all-reduce change the summation order, so the result is not
bit-identical to the sequential fold; it is within 1e-5 normwise of it (``tests/
test_ps_shard.py`` against ``oracle.ps_fedavg``; the per-call drop-in PS,
``consensus/_ps.py``, stays bit-exact with the sequential kernel).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple  # noqa: F401

import torch


def fedavg_coefficients(active: Sequence[int], update_factor: float,
                        ended: Optional[Sequence[int]] = None) -> Tuple[float, Dict[int, float]]:
    """(c_p, {device: c_k}) of the closed form of the reference's fold over ``active`` (device
    ids in the order the reference folds them). ``ended``: devices that reported training_end;
    if any of them is active, the transfer-learning branch applies to the first one in fold
    order (``parameter_server_v2.py:150-157``)."""
    active = list(active)
    u = float(update_factor)
    if ended:
        ended_set = set(ended)
        first = next((g for g in active if g in ended_set), None)
        if first is not None:
            return 1.0 - u, {first: u}
    C = len(active)
    if C == 0:
        return 1.0, {}
    a = u / C
    c_p = (1.0 - a) ** C
    return c_p, {g: a * (1.0 - a) ** (C - 1 - k) for k, g in enumerate(active)}


def device_block(rank: int, world: int, devices: int) -> Tuple[int, int]:
    """[first, last) of the contiguous device block of ``rank`` (blocks differ by at most one)."""
    return rank * devices // world, (rank + 1) * devices // world


class ShardedFedAvg:
    """One rank's share of a sharded parameter-server round.

    ``models`` [L, P] holds the models of this rank's devices [first, last); ``params`` [P] is
    the global model, replicated on every rank. ``aggregate`` replaces ``params`` with the
    aggregated global model (on every rank, or on ``reduce_to`` only)."""

    def __init__(self, rank: int, world: int, devices: int, P: int, device, transport=None, engine=None,
                 update_factor: float = 1.0, dtype=torch.float32):
        if devices < 1 or P < 0:
            raise ValueError("need at least one device and P >= 0")
        if world > 1 and transport is None:
            raise ValueError("a sharded aggregation needs a transport for world > 1")
        self.rank, self.world, self.devices, self.P = int(rank), int(world), int(devices), int(P)
        self.first, self.last = device_block(self.rank, self.world, self.devices)
        self.device = torch.device(device)
        self.transport, self.engine = transport, engine
        self.update_factor = float(update_factor)
        self.models = torch.empty((self.last - self.first, self.P), dtype=dtype, device=self.device)
        self.params = torch.empty(self.P, dtype=dtype, device=self.device)
        self._acc = torch.empty(self.P, dtype=dtype, device=self.device)

    def local_terms(self, active: Sequence[int], ended: Optional[Sequence[int]] = None):
        """(local bucket, neighbour buckets, coefficients) of this rank's pre-scaled partial sum,
        or None when the rank contributes nothing. Rank 0 carries the c_p * params term."""
        c_p, coef = fedavg_coefficients(active, self.update_factor, ended)
        mine = [g for g in coef if self.first <= g < self.last]  # fold order
        rows = [self.models[g - self.first] for g in mine]
        cs = [coef[g] for g in mine]
        if self.rank == 0:
            return self.params, rows, [c_p] + cs
        if not rows:
            return None
        return rows[0], rows[1:], cs

    def aggregate(self, active: Optional[Sequence[int]] = None, ended: Optional[Sequence[int]] = None,
                  stream=None, reduce_to: Optional[int] = None) -> torch.Tensor:
        """One aggregation round over the ``active`` devices (default: all, in device order).
        Enqueued on ``stream``; returns the new ``params``."""
        if active is None:
            active = range(self.devices)
        active = list(active)
        if any(not (0 <= g < self.devices) for g in active) or len(set(active)) != len(active):
            raise ValueError("active devices must be distinct ids in [0, devices)")
        terms = self.local_terms(active, ended)
        if terms is None:
            if stream is not None and self._acc.is_cuda:
                with torch.cuda.stream(stream):
                    self._acc.zero_()
            else:
                self._acc.zero_()
        else:
            local, nbrs, coeff = terms
            self.engine.mix_linear(self._acc, local, list(nbrs), [float(c) for c in coeff], stream=stream)
        if self.world > 1:
            if reduce_to is None:
                self.transport.allreduce_sum(self._acc, stream)
            else:
                self.transport.reduce_sum(self._acc, int(reduce_to), stream)
        if reduce_to is None or self.rank == reduce_to:
            self.params, self._acc = self._acc, self.params
        return self.params

    @property
    def bytes_per_round(self) -> int:
        """Algorithmic HBM bytes of this rank's pre-scaling pass: its models and the global model
        read once, the partial written once (the all-reduce's traffic is RCCL's)."""
        n = self.last - self.first
        return (n + (2 if self.rank == 0 else 1)) * self.P * self.models.element_size()
