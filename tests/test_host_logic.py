"""CPU tests of the product's host logic (no GPU): neighbour selection against the reference's
golden lists, bucket packing, the ring-shard plan, and the sharded halo exchange with the gloo
backend at world_size 2 (the N > 1 path's logic), checked against the unsharded oracle."""
import os
import random

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden, ragged


def test_product_topology_matches_reference_golden():
    from federated_amd.consensus import _tf1, _tf2
    z = load_golden("topology_kregular.npz")
    fns = {"tf1": _tf1.kregular, "v3": _tf2.kregular_v3, "v4": _tf2.kregular_ring, "v4tx": _tf2.tx_ring}
    for name, fn in fns.items():
        for (K, N, ii), expect in ragged(z[f"{name}_keys"], z[f"{name}_len"], z[f"{name}_vals"]).items():
            assert np.atleast_1d(fn(ii, N, K)).tolist() == expect, (name, K, N, ii)


def test_product_mobile_topology_matches_reference_golden(tmp_path, monkeypatch):
    import scipy.io as sio
    from federated_amd.consensus import _tf1
    z = load_golden("topology_mobile.npz")
    monkeypatch.chdir(tmp_path)
    os.makedirs("consensus")
    sio.savemat("consensus/vGraph.mat", {"graph": z["graph"]})
    for (g, ii, mx, seed), expect in ragged(z["mn_keys"], z["mn_len"], z["mn_vals"]).items():
        random.seed(seed)
        assert _tf1.mobile_neighbors(ii, mx, 5, g).tolist() == expect
    for (g, ii), expect in ragged(z["v3_keys"], z["v3_len"], z["v3_vals"]).items():
        assert _tf1.graph_row(ii, 5, g).tolist() == expect


def test_weight_factor_matches_reference_expression():
    from federated_amd.consensus import _tf1
    from oracle import cfa_oracle as O
    for devices in (5, 16, 80):
        for m in (0, 1, 2, 3):
            assert _tf1.weight_factor(devices, 1, 2, m) == float(O.tf1_weight_factor(devices, 1, 2, m))


def test_bucket_layout_roundtrip():
    from federated_amd.engine import BucketLayout
    rng = np.random.default_rng(0)
    arrays = [rng.standard_normal(s).astype(np.float32) for s in [(3, 3, 1, 4), (4,), (4096, 6), (6,)]]
    lay = BucketLayout.of(arrays)
    assert lay.P == 24622 and lay.segment(2) == (40, 40 + 24576)
    flat = lay.pack(arrays)
    for a, b in zip(lay.unpack(flat), arrays):
        assert np.array_equal(a, b)
    # biases coming back from .mat files are (1, m): same element count packs the same
    arrays2 = [arrays[0], arrays[1][None, :], arrays[2], arrays[3][None, :]]
    assert np.array_equal(lay.pack(arrays2), flat)
    with pytest.raises(ValueError):
        lay.pack(arrays[:3])


@pytest.mark.parametrize("world,L,hl,hr", [(1, 8, 2, 2), (2, 8, 4, 4), (4, 6, 3, 3), (8, 64, 4, 4),
                                           (3, 5, 2, 2), (8, 16, 1, 0), (4, 8, 2, 1)])
def test_ring_shard_plan(world, L, hl, hr):
    from federated_amd.population import RingShardPlan
    D = world * L
    for r in range(world):
        p = RingShardPlan(r, world, L, hl, hr)
        for i in range(L):
            g = p.first + i
            nb = p.neighbours(g)
            assert len(nb) == hl + hr and g not in nb and len(set(nb)) == hl + hr
            assert nb == [(g + o) % D for o in list(range(-hl, 0)) + list(range(1, hr + 1))]
            for j in nb:
                where, row = p.locate(j)
                if where == "local":
                    assert p.first + row == j
                elif where == "left":
                    assert (p.first - hl + row) % D == j
                else:
                    assert (p.first + L + row) % D == j
            remote = any(p.locate(j)[0] != "local" for j in nb)
            assert remote or not p.needs_halo(i) or world == 1
        assert sorted(p.interior() + p.boundary()) == list(range(L))


def _gloo_worker(rank, world, port, L, h, P, q, hr=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from federated_amd.population import RingPopulationShard, RingShardPlan
        from oracle.cfa_oracle import sequential_mix
        plan = RingShardPlan(rank, world, L, h, hr)
        shard = RingPopulationShard(plan, P, "cpu", TorchTransport())
        for i in range(L):
            g = torch.Generator().manual_seed(1000 + plan.first + i)
            shard.models[i] = torch.randn(P, generator=g)
        shard.exchange()
        D = plan.D
        allb = [torch.randn(P, generator=torch.Generator().manual_seed(1000 + g)).numpy() for g in range(D)]
        ok = True
        for i in range(L):
            g = plan.first + i
            srcs = [s.numpy() for s in shard.sources(i)]
            ok &= all(np.array_equal(s, allb[j]) for s, j in zip(srcs, plan.neighbours(g)))
            got = sequential_mix(shard.models[i].numpy(), srcs, shard.alphas)
            ref = sequential_mix(allb[g], [allb[j] for j in plan.neighbours(g)], shard.alphas)
            ok &= np.array_equal(got, ref)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,L,h,hr", [(2, 8, 4, 4), (2, 5, 2, 2), (3, 4, 2, 2),
                                          (8, 16, 1, 0),   # config 5: ring (v4 N=1), 128 devices / 8
                                          (4, 8, 2, 2)])   # config 4: 32 devices, K=4, 4 shards
def test_sharded_population_exchange_gloo(world, L, h, hr):
    """Multi-process (gloo) check of the N > 1 path: halo exchange places every remote
    neighbour bucket where the mix reads it, and each shard's mixes equal the unsharded
    population's (oracle on both sides)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + world * 7 + L
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, L, h, 1000, q, hr)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}
