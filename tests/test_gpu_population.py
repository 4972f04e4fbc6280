"""GPU tests of the population round, the RCCL transport owned by libcfa (world_size 1: grouped
self send/recv + all-reduce through the C-ABI) and the host-staging path."""
import numpy as np
import pytest
import torch

from oracle.cfa_oracle import sequential_mix

pytestmark = pytest.mark.gpu


def test_ring_population_round_world1(gpu):
    from federated_amd.population import RingPopulationShard, RingShardPlan
    plan = RingShardPlan(0, 1, 12, 4)
    shard = RingPopulationShard(plan, 50_003, torch.device("cuda"), None, gpu)
    shard.models.normal_()
    shard.round()
    torch.cuda.synchronize()
    host = shard.models.cpu().numpy()
    mixed = shard.mixed.cpu().numpy()
    for i in range(plan.L):
        ref = sequential_mix(host[i], [host[j] for j in plan.neighbours(i)], shard.alphas)
        assert np.array_equal(mixed[i], ref), i


def test_rccl_transport_world1():
    from federated_amd.dist import RcclTransport
    t = RcclTransport(0, 1, 0)
    try:
        a = torch.randn(100_003, device="cuda")
        b = torch.empty_like(a)
        c = torch.randn(7, device="cuda")
        d = torch.empty_like(c)
        t.exchange([(a, 0)], [(b, 0)])
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        with pytest.raises(ValueError):
            t.exchange([(a, 0)], [(d, 0)])
        ref = c.clone()
        t.allreduce_sum(c)
        torch.cuda.synchronize()
        assert torch.equal(c, ref)
    finally:
        t.close()


def test_population_shard_with_rccl_transport_world1(gpu):
    """world_size 1 never exchanges; the transport object is accepted and idle."""
    from federated_amd.dist import RcclTransport
    from federated_amd.population import RingPopulationShard, RingShardPlan
    t = RcclTransport(0, 1, 0)
    try:
        plan = RingShardPlan(0, 1, 10, 2)
        shard = RingPopulationShard(plan, 4096, torch.device("cuda"), t, gpu)
        shard.models.normal_()
        shard.round()
        torch.cuda.synchronize()
        h = shard.models.cpu().numpy()
        assert np.array_equal(shard.mixed[3].cpu().numpy(),
                              sequential_mix(h[3], [h[j] for j in plan.neighbours(3)], shard.alphas))
    finally:
        t.close()


def test_host_staging_e2e_small(gpu):
    from federated_amd.staging import measure_e2e
    r = measure_e2e(gpu, 1_000_003, 4, reps=2, chunks=4)
    assert r["pipelined_equals_device_result"]
    assert r["serial"]["ms"] > 0 and r["h2d_GBps"] > 0
