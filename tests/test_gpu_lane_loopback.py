"""The host lane on the exchange-first round, the order a real (RCCL) run takes.

The two-process lane tests go through gloo, whose host-staged exchange makes `population.round`
enqueue the interior mixes first (`host_staged`). On a multi-GPU node the transport is RCCL, which
only enqueues, so the round issues the exchange (and the lane's D2H side) first and the pump
threads feed the H2D side while the host enqueues the mixes. Here the ranks are host threads of
one process on the one GPU (tests/loopback.py: device-to-device copies with cfa_p2p_group_f32's
pairing, not host-staged), each with its own host lane (real shared-memory segments, pinned, one
pump thread per lane, its own lane streams), the route planned on rates that put part of the halo
on the lane; several rounds with the mixed models fed back, every device bit for bit against the
unsharded oracle trajectory. Worlds 2 (one pair, both halos), 4 and 8 (the bench's N = 8 plan: relays and
the lane together), and the hybrid partition at world 4 (2 device blocks x 2 element slices).
"""
import threading

import numpy as np
import pytest
import torch

from oracle.cfa_oracle import sequential_mix

pytestmark = pytest.mark.gpu


class _Agree:
    """All-ranks AND over the in-process rank threads (what the control plane gives a real run)."""

    def __init__(self, n):
        self.bar = threading.Barrier(n, timeout=120)
        self.vals = [True] * n

    def of(self, rank):
        def agree(ok):
            self.vals[rank] = bool(ok)
            self.bar.wait()
            res = all(self.vals)
            self.bar.wait()
            return res
        return agree


@pytest.mark.parametrize("world,D,P,partition", [(2, 32, 300_037, "devices"), (4, 64, 200_003, "devices"),
                                                 (8, 128, 100_003, "devices"), (4, 32, 200_003, "hybrid")])
def test_lane_exchange_first_round_matches_the_oracle(gpu, monkeypatch, world, D, P, partition):
    from loopback import LoopbackHub, run_ranks
    from federated_amd import hostlane, streams
    from federated_amd.halo import LANE_IN, LANE_OUT
    from federated_amd.population import make_ring_shard
    h, rounds = 4, 3
    full = [torch.randn(P, generator=torch.Generator().manual_seed(8100 + g)).numpy() for g in range(D)]
    rates = {(a, b): 50.0 for a in range(world) for b in range(world) if a != b}
    rates.update({(a, LANE_OUT): 50.0 for a in range(world)})
    rates.update({(LANE_IN, a): 50.0 for a in range(world)})
    # one process hosts every rank here: each rank thread gets lane streams of its own, as each
    # rank process of a real run does (streams.role_stream is per process)
    local = threading.local()
    real_role = streams.role_stream

    def per_thread_role(role, device=None):
        s = getattr(local, role, None)
        if s is None:
            s = torch.cuda.Stream()
            setattr(local, role, s)
        return s
    monkeypatch.setattr(streams, "role_stream", per_thread_role)
    agree = _Agree(world)
    token = hostlane.new_token()

    def rank_fn(rank, transport):
        assert not getattr(transport, "host_staged", False)  # the exchange-first order
        shard, info = make_ring_shard(rank, world, D, h, h, P, torch.device("cuda"), transport, gpu,
                                      partition=partition, dev_groups=2 if partition == "hybrid" else None,
                                      link_rates=rates, lane_token=token, lane_agree=agree.of(rank),
                                      lane_chunk_elems=1 << 14)
        lo, hi = info["slice"]
        try:
            cs, ms = torch.cuda.Stream(), torch.cuda.Stream()
            with torch.cuda.stream(cs):
                for i in range(shard.plan.L):
                    shard.models[i].copy_(torch.from_numpy(full[shard.plan.first + i][lo:hi]))
                for _ in range(rounds):
                    shard.round(cs, ms)
                    shard.models.copy_(shard.mixed)
            cs.synchronize()
            return (shard.plan.first, shard.models.cpu().numpy(), info["route"]["lane"], info["route"]["lane_elems"],
                    (lo, hi))
        finally:
            shard.close()

    hub = LoopbackHub(world)
    res = run_ranks(world, rank_fn, hub=hub)
    assert streams.role_stream is per_thread_role and real_role is not per_thread_role
    assert all(r[2] for r in res) and res[0][3] > 0  # the plan put pieces on the lane
    assert sum(hub.messages) > 0 or world == 2  # and (at 4) on the loopback links too
    offs = list(range(-h, 0)) + list(range(1, h + 1))
    cur = [x.copy() for x in full]
    for _ in range(rounds):
        cur = [sequential_mix(cur[d], [cur[(d + o) % D] for o in offs], [1.0 / (2 * h + 1)] * (2 * h))
               for d in range(D)]
    for first, block, _, _, (lo, hi) in res:  # hybrid: each rank holds an element slice of its block
        for i in range(block.shape[0]):
            assert np.array_equal(block[i], cur[first + i][lo:hi]), first + i
