"""Sharding a population on an arbitrary topology (SURVEY §8 e): the CSR-driven halo plan
(GraphShardPlan) on CPU, and the N > 1 exchange with the gloo backend (world 2, 3, 4) against the
unsharded population mixed by the oracle."""
import multiprocessing as mp
import os
import random

import numpy as np
import pytest
import torch
import torch.distributed as dist

from federated_amd import topology as T
from federated_amd.graph_population import GraphShardPlan, block_bounds


def _random_graph(D, p, seed):
    rng = np.random.default_rng(seed)
    g = (rng.random((D, D)) < p).astype(np.uint8)
    g = np.maximum(g, g.T)
    np.fill_diagonal(g, 0)
    return g[:, :, None]


def _topologies():
    return {
        "kregular_tf1_32_4": T.kregular_tf1(32, 4),
        "kregular_v3_30_5": T.kregular_v3(30, 5),
        "ring_v4_16": T.ring_v4(16, 1),
        "vgraph_choices_40": T.mobile(_random_graph(40, 0.2, 1), 0, 3, rng=random.Random(7)),
        "vgraph_full_rows_24": T.mobile(_random_graph(24, 0.3, 2), 0),
    }


@pytest.mark.parametrize("name", sorted(_topologies()))
@pytest.mark.parametrize("world", [1, 2, 3, 4, 5])
def test_graph_plan_invariants(name, world):
    lists = _topologies()[name]
    D = len(lists)
    plans = [GraphShardPlan(lists, r, world) for r in range(world)]
    assert sum(p.L for p in plans) == D and block_bounds(D, world)[-1] == D
    for p in plans:
        for i in range(p.L):
            g = p.first + i
            for j in p.neighbours(g):  # every neighbour is local or in the halo
                where, row = p.locate(j)
                assert (where == "local") == (p.owner(j) == p.rank)
            assert p.needs_halo(i) == (i in p.boundary())
        assert sorted(p.interior() + p.boundary()) == list(range(p.L))
    # pairing: r's k-th send to q is q's k-th receive from r (same global device)
    for r, pr in enumerate(plans):
        sends, _ = pr.halo_transfers()
        for q, pq in enumerate(plans):
            if q == r:
                continue
            sent = [pr.first + row for row, peer in sends if peer == q]
            _, recvs = pq.halo_transfers()
            got = [pq.halo_devices[h] for h, peer in recvs if peer == r]
            assert sent == got, (r, q)


def _gloo_worker(rank, world, port, topo, P, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from federated_amd.graph_population import GraphPopulationShard
        from oracle.cfa_oracle import sequential_mix
        lists = _topologies()[topo]
        plan = GraphShardPlan(lists, rank, world)
        shard = GraphPopulationShard(plan, P, "cpu", TorchTransport())
        seed = lambda g: torch.Generator().manual_seed(500 + g)
        for i in range(plan.L):
            shard.models[i] = torch.randn(P, generator=seed(plan.first + i))
        shard.exchange()
        allb = [torch.randn(P, generator=seed(g)).numpy() for g in range(plan.D)]
        ok = True
        for i in range(plan.L):
            g = plan.first + i
            srcs = [s.numpy() for s in shard.sources(i)]
            ok &= all(np.array_equal(s, allb[j]) for s, j in zip(srcs, plan.neighbours(g)))
            got = sequential_mix(shard.models[i].numpy(), srcs, shard.alphas[i])
            ref = sequential_mix(allb[g], [allb[j] for j in plan.neighbours(g)], T.alphas_tf2(plan.neighbours(g), g, plan.D))
            ok &= np.array_equal(got, ref)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,topo", [(2, "vgraph_choices_40"), (3, "vgraph_full_rows_24"),
                                        (4, "kregular_v3_30_5"), (3, "ring_v4_16")])
def test_graph_sharded_exchange_gloo(world, topo):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31000 + (os.getpid() % 1000) + 11 * world + len(topo)
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, topo, 777, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}
