"""Sharded FedAvg / parameter-server rounds (federated_amd/ps_shard.py) on CPU with gloo.

Each rank pre-scales its own devices' models (the closed form of the reference's sequential
fold, parameter_server_v2.py:159-161) and one sum all-reduce (or reduce to the owner) forms the
new global model. The summation order differs from the reference's, so the bar is 1e-5
normwise against oracle.ps_fedavg (the sequential fold), per SURVEY §8(c)'s tolerance. A stub
engine stands in for cfa_mix_f32 here (no GPU); the GPU test (test_gpu_population.py) runs the
real kernel.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from federated_amd.ps_shard import ShardedFedAvg, device_block, fedavg_coefficients

TOL = 1e-5


class LinearStub:
    """cfa_mix_f32's linear rule on CPU tensors (fp32 multiply-adds, left to right)."""

    @staticmethod
    def mix_linear(out, local, nbrs, coeff, stream=None):
        acc = torch.tensor(coeff[0], dtype=torch.float32) * local
        for c, x in zip(coeff[1:], nbrs):
            acc = acc + torch.tensor(c, dtype=torch.float32) * x
        out.copy_(acc)


def _models(D, P, seed=5):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(P).astype(np.float32) for _ in range(D)], rng.standard_normal(P).astype(np.float32)


def _normwise(got, ref):
    return float(np.max(np.abs(got - ref)) / np.max(np.abs(ref)))


def test_coefficients_equal_the_sequential_fold():
    from oracle.cfa_oracle import ps_fedavg
    for C, u in [(1, 1.0), (4, 1.0), (7, 0.99), (32, 0.5)]:
        c_p, coef = fedavg_coefficients(range(C), u)
        xs = [np.float64(k + 2.0) for k in range(C)]
        seq = ps_fedavg([np.float64(1.0)], [[x] for x in xs], u)[0]
        closed = c_p * 1.0 + sum(coef[k] * xs[k] for k in range(C))
        assert abs(seq - closed) <= 1e-12 * abs(seq)
    c_p, coef = fedavg_coefficients([3, 1, 2], 0.9, ended=[2, 1])
    assert c_p == pytest.approx(0.1) and coef == {1: 0.9}  # first ended device in fold order


def test_device_blocks_cover_the_population():
    for D, W in [(8, 2), (10, 3), (128, 8), (5, 8)]:
        spans = [device_block(r, W, D) for r in range(W)]
        assert spans[0][0] == 0 and spans[-1][1] == D
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _worker(rank, world, port, D, P, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from oracle.cfa_oracle import ps_fedavg
        models, params = _models(D, P)
        u = 0.99 if case != "all" else 1.0
        ps = ShardedFedAvg(rank, world, D, P, "cpu", TorchTransport(), LinearStub(), update_factor=u)
        for i in range(ps.last - ps.first):
            ps.models[i] = torch.from_numpy(models[ps.first + i])
        ps.params.copy_(torch.from_numpy(params))
        active, ended, reduce_to = None, None, None
        if case == "subset":
            active = [g for g in range(D) if g % 3 != 1]
        elif case == "ended":
            active, ended = list(range(D)), [D - 2, D - 1]
        elif case == "reduce":
            reduce_to = world - 1
        out = ps.aggregate(active, ended, reduce_to=reduce_to).numpy()
        act = list(range(D)) if active is None else active
        if ended:
            e = next(g for g in act if g in ended)
            ref = params + u * (models[e] - params)
        else:
            ref = ps_fedavg([params], [[models[g]] for g in act], u)[0]
        err = _normwise(out, ref) if (reduce_to is None or rank == reduce_to) else 0.0
        q.put((rank, err))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,D,case", [(2, 8, "all"), (4, 32, "all"), (3, 10, "subset"), (4, 16, "ended"),
                                          (4, 12, "reduce"), (2, 3, "subset")])
def test_sharded_fedavg_gloo(world, D, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    P = 2000 + 17
    port = 34000 + (os.getpid() % 911) + world * 13 + D + 3 * len(case)
    procs = [ctx.Process(target=_worker, args=(r, world, port, D, P, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    errs = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert sorted(errs) == list(range(world))
    assert max(errs.values()) <= TOL, errs
