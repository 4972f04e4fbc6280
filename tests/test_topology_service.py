"""Topology service (f4): CSR tables built from the reference's rules (pinned by the golden
neighbour lists), and one-launch population rounds against per-device oracle mixes (GPU)."""
import random

import numpy as np
import pytest
import torch

from conftest import load_golden, ragged
from oracle import cfa_oracle as O


def test_lists_match_reference_golden():
    from federated_amd import topology as T
    z = load_golden("topology_kregular.npz")
    for name, fn in (("tf1", T.kregular_tf1), ("v3", T.kregular_v3), ("v4", T.ring_v4)):
        table = ragged(z[f"{name}_keys"], z[f"{name}_len"], z[f"{name}_vals"])
        for K in (5, 8, 16, 32, 128):
            for N in (1, 2, 3, 4):
                lists = fn(K, N)
                assert [table[(K, N, ii)] for ii in range(K)] == lists, (name, K, N)


def test_mobile_lists_match_reference_random_draws():
    from federated_amd import topology as T
    z = load_golden("topology_mobile.npz")
    table = ragged(z["mn_keys"], z["mn_len"], z["mn_vals"])
    graph = z["graph"]
    for g in range(0, graph.shape[2], 7):
        for mx in (1, 2, 3, 4):
            for ii in range(5):  # golden draws were seeded per (g, ii, mx)
                random.seed(g * 1000 + ii * 10 + mx)
                nb = O.mobile_neighbors(graph, ii, mx, 5, g).tolist()
                assert nb == table[(g, ii, mx, g * 1000 + ii * 10 + mx)]
        random.seed(123)
        lists = T.mobile(graph, g, 2)
        random.seed(123)
        assert lists == [O.mobile_neighbors(graph, ii, 2, 5, g).tolist() for ii in range(5)]


def test_csr_tables_policies():
    from federated_amd import topology as T
    lists = T.kregular_tf1(8, 3)
    ptr, idx, coef = T.csr(lists, T.alphas_tf1_cfa(0.7, 3))
    assert ptr[0] == 0 and ptr[-1] == len(idx) == len(coef) == 8 + sum(len(l) for l in lists)
    for d in range(8):
        row = idx[ptr[d]:ptr[d + 1]].tolist()
        assert row == [d] + lists[d]
        a = coef[ptr[d] + 1:ptr[d + 1]]
        assert np.allclose(a, [0.7 * float(O.tf1_weight_factor(8, d, j, 2)) for j in lists[d]])
    _, _, c2 = T.csr([[1, 2]], T.alphas_tf2)
    assert c2.tolist() == [1.0, np.float32(1 / 3), np.float32(1 / 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("rule", ["tf1_cfa", "tf1_ongraphs", "tf2"])
def test_population_round_matches_per_device_calls(gpu, rule):
    from federated_amd import topology as T
    D, P = 16, 200_003
    models = torch.randn(D, P, device="cuda")
    pr = T.PopulationRound(gpu, models)
    if rule == "tf1_cfa":
        lists, pol = T.kregular_tf1(D, 3), T.alphas_tf1_cfa(1.0, 3)
    elif rule == "tf1_ongraphs":
        lists, pol = T.kregular_tf1(D, 2), T.alphas_tf1_ongraphs(0.8)
    else:
        lists, pol = T.ring_v4(D, 1), T.alphas_tf2
    pr.set_topology(lists, pol)
    out = pr.run()
    torch.cuda.synchronize()
    host = models.cpu().numpy()
    for d in range(D):
        a = [float(np.float32(x)) for x in pol(lists[d], d, D)]
        ref = O.sequential_mix(host[d], [host[j] for j in lists[d]], a)
        assert np.array_equal(out[d].cpu().numpy(), ref), (rule, d)


def test_window_shape_detection():
    from federated_amd import topology as T
    win = lambda D, hl, hr: [[(d + o) % D for o in list(range(-hl, 0)) + list(range(1, hr + 1))] for d in range(D)]
    pol = lambda lists, p: [p(nb, d, len(lists)) for d, nb in enumerate(lists)]
    assert T.window_shape(T.ring_v4(16, 1), pol(T.ring_v4(16, 1), T.alphas_tf2)) == (1, 0)
    assert T.window_shape(win(32, 2, 2), pol(win(32, 2, 2), T.alphas_tf2)) == (2, 2)
    assert T.window_shape(win(20, 4, 4), pol(win(20, 4, 4), T.alphas_tf2)) == (4, 4)
    assert T.window_shape(win(20, 0, 3), pol(win(20, 0, 3), T.alphas_tf2)) == (0, 3)
    # clamped k-regular windows (edges shift) and wider windows stay on the CSR kernel
    assert T.window_shape(T.kregular_v3(30, 4), pol(T.kregular_v3(30, 4), T.alphas_tf2)) is None
    assert T.window_shape(T.kregular_tf1(32, 4), pol(T.kregular_tf1(32, 4), T.alphas_tf2)) is None
    assert T.window_shape(win(40, 5, 5), pol(win(40, 5, 5), T.alphas_tf2)) is None
    # step-varying coefficients cannot use the one-alpha-per-device window pass
    lists = win(16, 1, 1)
    assert T.window_shape(lists, [[0.5, 0.25]] * 16) is None


@pytest.mark.gpu
@pytest.mark.parametrize("P", [200_003, 1_488])
@pytest.mark.parametrize("rule", ["tf1_cfa", "tf1_ongraphs"])
def test_population_round_tf1_numerics(gpu, rule, P):
    """numerics="tf1" (cfa_mix_population_tf1_f32): every device equals fp32 of the reference's
    numpy-2 chain (oracle.tf1_mix_flat: fp32 first subtraction, fp64 after) and the per-device
    cfa_mix_tf1_f32 launch, bit for bit; a device without neighbours keeps its model."""
    from federated_amd import topology as T
    D = 12
    models = torch.randn(D, P, device="cuda")
    pr = T.PopulationRound(gpu, models)
    if rule == "tf1_cfa":
        lists, pol = T.kregular_tf1(D, 3), T.alphas_tf1_cfa(0.9, 3)
    else:
        lists, pol = T.kregular_tf1(D, 2), T.alphas_tf1_ongraphs(0.8)
    lists[5] = []
    pr.set_topology(lists, pol, numerics="tf1")
    out = pr.run()
    torch.cuda.synchronize()
    host = models.cpu().numpy()
    one = torch.empty(P, device="cuda")
    for d in range(D):
        a = pol(lists[d], d, D)
        ref = np.asarray(O.tf1_mix_flat(host[d], [host[j] for j in lists[d]], a)).astype(np.float32)
        assert np.array_equal(out[d].cpu().numpy(), ref), (rule, d)
        if lists[d]:
            gpu.mix_tf1(one, models[d], [models[j] for j in lists[d]], a)
            torch.cuda.synchronize()
            assert torch.equal(one, out[d]), (rule, d)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3, 4])
def test_population_round_tf1_compression(gpu, mode):
    """BASELINE config 2 as one population launch: FL_CFA_CNN_tf2 buckets (P = 24 622, W2 =
    elements [44, 24620)), 8 devices, 3 neighbours, the cfa_ongraphs alpha eps/(1+n), and the
    compression epilogue on W2 (cfa_ongraphs.py:225-273). Every device equals the per-device
    cfa_mix_tf1_f32 launch bit for bit, counter_param included; a device without neighbours gets
    the fp32 epilogue on its own model, as the reference compresses the caller's array."""
    from federated_amd import topology as T
    D, P, cb, ce = 8, 24_624, 44, 44 + 4096 * 6
    g = torch.Generator(device="cuda").manual_seed(mode)
    scale = {1: 1e-3, 2: 1e-4, 3: 1e-3, 4: 1e-2}[mode]  # weights near each mode's threshold
    models = torch.randn(D, P, device="cuda", generator=g) * scale
    lists = [[(d + o) % D for o in (-1, 1, 2)] for d in range(D)]
    lists[3] = []
    pol = T.alphas_tf1_ongraphs(0.8)
    pr = T.PopulationRound(gpu, models)
    pr.set_topology(lists, pol, numerics="tf1", compression=(mode, cb, ce))
    out = pr.run()
    torch.cuda.synchronize()
    one = torch.empty(P, device="cuda")
    kept = torch.zeros(1, dtype=torch.int64, device="cuda")
    for d in range(D):
        kept.zero_()
        gpu.mix_tf1(one, models[d], [models[j] for j in lists[d]], pol(lists[d], d, D), mode, cb, ce, kept)
        torch.cuda.synchronize()
        assert torch.equal(one, out[d]), (mode, d)
        assert int(kept.item()) == int(pr.kept[d].item()), (mode, d)
    assert 0 < int(pr.kept.sum().item()) < D * (ce - cb)
