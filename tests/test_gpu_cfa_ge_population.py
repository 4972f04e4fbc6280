"""Device-resident CFA-GE population (BASELINE config 3, cfa_ge_2stage.py:388-621 for every
device) against the oracle's float64 composition of the reference's per-device steps
(oracle.cfa_ge_population_round), over several rounds: within 1e-5 normwise per device bucket."""
import numpy as np
import pytest
import torch

from conftest import normwise_close
from oracle import cfa_oracle as orc

pytestmark = pytest.mark.gpu

CNN = {"filter": 16, "number": 8, "stride": 5, "input_data": 512, "classes": 8}
NN2 = {"intermediate_nodes": 32, "input_data": 512, "classes": 8}


@pytest.mark.parametrize("ml,D,N", [(1, 16, 2), (2, 16, 2), (1, 7, 3), (2, 5, 4)])
def test_population_rounds_match_oracle(gpu, ml, D, N):
    from federated_amd import topology
    from federated_amd.cfa_ge_population import CfaGePopulation
    geom = CNN if ml == 1 else NN2
    rng = np.random.default_rng(D * 10 + N + ml)
    lists = topology.kregular_tf1(D, N)
    shapes = orc.tf1_flat_shapes(ml, geom)
    P = sum(int(np.prod(s)) for s in shapes)
    B = 24
    x = rng.standard_normal((D, B, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[rng.integers(0, 8, (D, B))]
    W = (rng.standard_normal((D, P)) * 0.1).astype(np.float32)
    pub = (rng.standard_normal((D, P)) * 0.1).astype(np.float32)
    Nmax = max(len(l) for l in lists)
    S = (rng.standard_normal((D, Nmax, P)) * 0.01).astype(np.float32)
    G = (rng.standard_normal((D, Nmax, P)) * 0.01).astype(np.float32)
    pop = CfaGePopulation(gpu, ml, {k: v for k, v in geom.items() if k not in ("input_data", "classes")},
                          torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), lists, eps=1.0, neighbors=N,
                          rho=0.99, lr1=0.1, lr2=0.1)
    pop.load(torch.from_numpy(W).cuda(), torch.from_numpy(pub).cuda(), torch.from_numpy(S).cuda(),
             torch.from_numpy(G).cuda())
    rW, rpub, rS, rG = W.astype(np.float64), pub.astype(np.float64), S.astype(np.float64), G.astype(np.float64)
    for _ in range(3):
        pop.round()
        rW, rS, rG, rpub = orc.cfa_ge_population_round(rW, rpub, rG, rS, lists, x, y, ml, geom, 1.0, N, 0.99, 0.1, 0.1)
        torch.cuda.synchronize()
        gW, gpub = pop.W.cpu().numpy(), pop.pub.cpu().numpy()
        gS, gG = pop.S.cpu().numpy(), pop.G.cpu().numpy().reshape(D, Nmax, P)
        for i in range(D):
            assert normwise_close(gW[i], rW[i]), ("W", i)
            assert normwise_close(gpub[i], rpub[i]), ("pub", i)
            for n in range(len(lists[i])):
                assert normwise_close(gS[i, n], rS[i, n]), ("S", i, n)
                assert normwise_close(gG[i, n], rG[i, n]), ("G", i, n)
        # carry the GPU state forward so rounding differences do not compound in the comparison
        rW, rpub, rS, rG = gW.astype(np.float64), gpub.astype(np.float64), gS.astype(np.float64), gG.astype(np.float64)


@pytest.mark.parametrize("P,filtered,wide", [(1488, True, False), (1001, False, False), (7, True, False),
                                             (1488, True, True), (1001, False, True)])
def test_fused_step_equals_mix_then_mewma(gpu, P, filtered, wide):
    """cfa_ge_population_step_f32 == cfa_mix_population_f32 followed by cfa_mewma_update_f32,
    bit for bit (separate 16-byte-aligned allocations so P % 4 != 0 exercises the tail; one
    neighbour slot without gradients)."""
    from federated_amd import _lib
    D = 4
    # wide: a device with 7 neighbours (longer fold and gradient chains)
    lists = [[1, 2, 3, 0, 2, 3, 1] if wide else [1, 2], [0], [3, 0, 1], []]
    g = torch.Generator(device="cuda").manual_seed(P)
    rnd = lambda: torch.randn(P, device="cuda", generator=g)
    W = [rnd() for _ in range(D)]
    pub = [rnd() for _ in range(D)]
    S = [[rnd() for _ in nb] for nb in lists]
    S2 = [[t.clone() for t in row] for row in S]
    G = [[rnd() if (i + n) % 3 else None for n in range(len(nb))] for i, nb in enumerate(lists)]
    out1 = [torch.empty(P, device="cuda") for _ in range(D)]
    out2 = [torch.empty(P, device="cuda") for _ in range(D)]
    ptr, idx, coef, states, grads = [0], [], [], [], []
    for i, nb in enumerate(lists):
        idx.append(i), coef.append(0.0), states.append(0), grads.append(0)
        for n, j in enumerate(nb):
            idx.append(D + j), coef.append(0.25 + 0.1 * n)
            states.append(S[i][n].data_ptr())
            grads.append(G[i][n].data_ptr() if G[i][n] is not None else 0)
        ptr.append(len(idx))
    t = lambda v, dt: torch.tensor(v, dtype=dt, device="cuda")
    src = t([w.data_ptr() for w in W] + [p.data_ptr() for p in pub], torch.int64)
    tabs = (t(ptr, torch.int32), t(idx, torch.int32), t(coef, torch.float32))
    gpu.ge_population_step(t([o.data_ptr() for o in out1], torch.int64), src, t(states, torch.int64),
                           t(grads, torch.int64), *tabs, D, 0.99, 0.1, 0.05, 5, filtered, P)
    gpu.population(t([o.data_ptr() for o in out2], torch.int64), src, *tabs, D, _lib.RULE_SEQUENTIAL, P)
    zero = torch.zeros(P, device="cuda")
    for i, nb in enumerate(lists):
        if nb:
            gpu.mewma(out2[i], S2[i], [x if x is not None else zero for x in G[i]], 0.99, 0.1, 0.05, 5, False, filtered)
    torch.cuda.synchronize()
    for i in range(D):
        assert torch.equal(out1[i], out2[i]), i
        for n in range(len(lists[i])):
            assert torch.equal(S[i][n], S2[i][n]), (i, n)


@pytest.mark.parametrize("ml", [1, 2])
def test_partials_reduced_in_step_launch_equal_rows_reduction(gpu, ml):
    """A partials-only gradient launch summed by cfa_ge_population_step_f32's reduction rows
    equals the rows launch's own reduction bit for bit, and the step's outputs are unchanged by
    the extra rows."""
    from federated_amd import topology
    rng = np.random.default_rng(77 + ml)
    D, N, B = 16, 2, 24
    geom = {"filter": 16, "number": 8, "stride": 5} if ml == 1 else {"intermediate_nodes": 32}
    full = {**geom, "input_data": 512, "classes": 8}
    P = sum(int(np.prod(s)) for s in orc.tf1_flat_shapes(ml, full))
    lists = topology.kregular_tf1(D, N)
    x = torch.from_numpy(rng.standard_normal((D, B, 512)).astype(np.float32)).cuda()
    y = torch.from_numpy(np.eye(8, dtype=np.float32)[rng.integers(0, 8, (D, B))]).cuda()
    models = torch.from_numpy((rng.standard_normal((D, P)) * 0.1).astype(np.float32)).cuda()
    mrow = torch.tensor([j for nb in lists for j in nb], dtype=torch.int32, device="cuda")
    drow = torch.tensor([i for i, nb in enumerate(lists) for _ in nb], dtype=torch.int32, device="cuda")
    M = mrow.numel()
    Sp = gpu.grad_splits(M, B, P)
    assert Sp > 1
    ref = torch.empty(M, P, device="cuda")
    gpu.grad_rows(ml, x, y, models, mrow, drow, ref, geom, workspace=gpu.grad_workspace(M, B, P))
    ws = torch.empty(M * Sp * P, device="cuda")
    gpu.grad_rows(ml, x, y, models, mrow, drow, None, geom, workspace=ws)
    # a small population step alongside the reduction
    t = lambda v, dt: torch.tensor(v, dtype=dt, device="cuda")
    W = torch.randn(2, P, device="cuda")
    S1, S2 = torch.randn(P, device="cuda"), None
    S2 = S1.clone()
    g = torch.randn(P, device="cuda")
    outs = [torch.empty(P, device="cuda") for _ in range(2)]
    src = t([W[0].data_ptr(), W[1].data_ptr()], torch.int64)
    tabs = (t([0, 2], torch.int32), t([0, 1], torch.int32), t([0.0, 0.4], torch.float32))
    got = torch.full((M, P), float("nan"), device="cuda")
    gpu.ge_population_step(t([outs[0].data_ptr()], torch.int64), src, t([0, S1.data_ptr()], torch.int64),
                           t([0, g.data_ptr()], torch.int64), *tabs, 1, 0.99, 0.1, 0.05, 5, True, P,
                           reduce=(ws, got, Sp))
    gpu.ge_population_step(t([outs[1].data_ptr()], torch.int64), src, t([0, S2.data_ptr()], torch.int64),
                           t([0, g.data_ptr()], torch.int64), *tabs, 1, 0.99, 0.1, 0.05, 5, True, P)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert torch.equal(outs[0], outs[1]) and torch.equal(S1, S2)
