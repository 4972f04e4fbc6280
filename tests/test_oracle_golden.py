"""Pin the CPU oracle (oracle/cfa_oracle.py) to the golden vectors produced by running the
reference code (tests/golden/make_golden.py). CPU-only; no GPU needed."""
import numpy as np
import pytest

from conftest import load_golden, ragged
from oracle import cfa_oracle as O


def test_topology_kregular_matches_reference():
    z = load_golden("topology_kregular.npz")
    fns = {"tf1": O.tf1_kregular, "v3": O.tf2_kregular_v3, "v4": O.tf2_kregular_v4, "v4tx": O.tf2_tx_v4}
    for name, fn in fns.items():
        table = ragged(z[f"{name}_keys"], z[f"{name}_len"], z[f"{name}_vals"])
        assert table, name
        for (K, N, ii), expect in table.items():
            got = np.atleast_1d(fn(ii, N, K)).tolist()
            assert got == expect, (name, K, N, ii)


def test_topology_mobile_matches_reference():
    import random
    z = load_golden("topology_mobile.npz")
    graph = z["graph"]
    table = ragged(z["mn_keys"], z["mn_len"], z["mn_vals"])
    for (g, ii, mx, seed), expect in table.items():
        random.seed(seed)
        assert O.mobile_neighbors(graph, ii, mx, 5, g).tolist() == expect, (g, ii, mx)


def _tf1_models(z, tag, prefix, dev):
    return [z[f"{tag}/{prefix}_{t}"][dev] for t in range(4)]


@pytest.mark.parametrize("tag", ["2nn_K5_N2_eps1", "2nn_K4_N2_eps1", "cnn_K5_N2_eps05", "cnn_K5_N3_eps1", "cnn_K8_N4_eps07"])
def test_tf1_cfa_oracle_bitexact(tag):
    z = load_golden("tf1_cfa.npz")
    K, N = (int(x) for x in z[f"{tag}/meta"])
    eps = float(z[f"{tag}/eps"])
    for ii in z[f"{tag}/under_test"]:
        ii = int(ii)
        nbr = O.tf1_kregular(ii, N, K)
        assert nbr.tolist() == z[f"{tag}/nbr_{ii}"].tolist()
        local = _tf1_models(z, tag, "e1", ii)
        nbrs = [_tf1_models(z, tag, "e0", int(j)) for j in nbr]
        wf = [O.tf1_weight_factor(K, ii, int(j), N - 1) for j in nbr]
        got = O.tf1_mix(local, nbrs, eps, wf)
        for t in range(4):
            ref = z[f"{tag}/out_{ii}_{t}"]
            assert got[t].dtype == ref.dtype and got[t].shape == ref.shape
            assert np.array_equal(got[t], ref), (tag, ii, t)


def test_tf1_ongraphs_oracle_bitexact():
    z = load_golden("tf1_ongraphs.npz")
    for tag in z["cases"]:
        tag = str(tag)
        ii, graph, mode, comp, ncalls = (int(x) for x in z[f"{tag}/meta"])
        kind = str(z[f"{tag}/kind"])
        eps = float(z[f"{tag}/eps"])
        prev_n = 1  # CFA_process.__init__ leaves self.neighbors = 1 (cfa_ongraphs.py:145-146)
        for c in range(ncalls):
            src = str(z[f"{tag}/call{c}_src"])
            local = [z[f"{kind}/{src}_{t}"][ii].copy() for t in range(4)]
            if graph == 0:
                nbr = O.tf1_kregular(ii, prev_n, 5)
            else:
                nbr = z[f"{tag}/call{c}_nbrs"] if not bool(z[f"{tag}/call{c}_stop"]) else np.zeros(0, np.int64)
            n = len(nbr)
            prev_n = n
            if n > 0:
                nbrs = [[z[f"{kind}/e0_{t}"][int(j)] for t in range(4)] for j in nbr]
                wf = [O.tf1_weight_factor(5, ii, int(j), n) for j in nbr]
                out = O.tf1_mix(local, nbrs, eps, wf)
            else:
                out = local  # aliasing: W_up_l2 IS the caller's n_W_l2
            counter = O.tf1_compress(out[2], local[2], comp)
            for t in range(4):
                ref = z[f"{tag}/call{c}_out_{t}"]
                assert np.array_equal(np.asarray(out[t]).reshape(ref.shape), ref), (tag, c, t)
            assert counter == int(z[f"{tag}/call{c}_counter"]), (tag, c)
            assert np.array_equal(local[2], z[f"{tag}/call{c}_in2_after"]), (tag, c)


@pytest.mark.parametrize("model", ["cnn", "2nn"])
@pytest.mark.parametrize("variant", ["fast", "4stage_e1", "4stage_e3"])
@pytest.mark.parametrize("ii", [0, 7])
def test_tf1_cfa_ge_oracle(model, variant, ii):
    z = load_golden("tf1_cfa_ge.npz")
    tag = f"{model}_{variant}_ii{ii}"
    K, N, ii_, epoch, ml = (int(x) for x in z[f"{tag}/meta"])
    rho, eps, lr1, lr2 = (float(x) for x in z[f"{tag}/hyper"])
    nbr = z[f"{tag}/nbr"]
    assert nbr.tolist() == O.tf1_kregular(ii, N, K).tolist()
    local = [z[f"{tag}/local_{t}"] for t in range(4)]
    prev = [[z[f"{tag}/prev{q}_{t}"] for t in range(4)] for q in range(len(nbr))]
    wf = [O.tf1_weight_factor(K, ii, int(j), N - 1) for j in nbr]
    W = O.tf1_mix(local, prev, eps, wf)
    states = [z[f"{tag}/state_in_{t}"].copy() for t in range(4)]
    # the fixtures hold the slot the reference reads, g[..., ii] (cfa_ge_2stage.py:575-589)
    grads = [[z[f"{tag}/grad{q}_{t}"] for t in range(4)] for q in range(len(nbr))]
    use_filtered = (variant == "fast" and ml == 1)
    init = variant == "4stage_e1"
    W = O.tf1_mewma(W, states, grads, rho, lr1, lr2, use_filtered, init)
    for t in range(4):
        ref = z[f"{tag}/out_{t}"]
        assert np.array_equal(np.asarray(W[t]).reshape(ref.shape), ref), (tag, t)
        assert np.array_equal(states[t], z[f"{tag}/state_out_{t}"]), (tag, "state", t)


def test_tf2_consensus_oracle_bitexact():
    z = load_golden("tf2_consensus.npz")
    L = 6
    models = [[z[f"models_{t}"][d] for t in range(L)] for d in range(z["models_0"].shape[0])]
    grads = [[z[f"grads_{t}"][d] for t in range(L)] for d in range(z["grads_0"].shape[0])]
    local = [z[f"local_{t}"] for t in range(L)]
    local_g = [z[f"local_g_{t}"] for t in range(L)]
    for tag in z["cases"]:
        tag = str(tag)
        nbr = z[f"{tag}/nbr"].tolist()
        ended = set(z[f"{tag}/ended"].tolist())
        eps = float(z[f"{tag}/eps"])
        # the reference stops loading after the first neighbour that reports training_end
        loaded = []
        end = False
        for j in nbr:
            loaded.append(j)
            end = j in ended
            if end:
                break
        if "_w_" in tag:
            out = O.tf2_weights(local, [models[j] for j in loaded], training_end=end)
        elif tag.startswith("v3"):
            out = O.tf2_grads_v3(local_g, [grads[j] for j in loaded])
        else:
            out = O.tf2_grads_v4(local_g, [grads[j] for j in loaded], eps)
        for t in range(L):
            ref = z[f"{tag}/out_{t}"]
            assert out[t].dtype == ref.dtype == np.float32
            assert np.array_equal(out[t], ref), (tag, t)
            assert np.array_equal(out[t], z[f"{tag}/inplace_{t}"]), (tag, t)
        assert bool(z[f"{tag}/meta"][1]) == end


def test_tf2_variant_copies_oracle_bitexact():
    """variants.npz: CIFAR-100 v3_threading, FL_over_MQTT v3 and FL_radar v4 (one neighbour id
    read ``neighbors`` times, FL_radar_dataset/consensus/consensus_v4.py:86-89) all reduce to the
    same weight rule (tf2_weights)."""
    z = load_golden("variants.npz")
    L = 6
    models = [[z[f"tf2/models_{t}"][d] for t in range(L)] for d in range(z["tf2/models_0"].shape[0])]
    local = [z[f"tf2/local_{t}"] for t in range(L)]
    for tag in (str(t) for t in z["tf2/cases"]):
        nbr = np.atleast_1d(z[f"tf2/{tag}/nbr"]).tolist()
        if tag.startswith("radar_v4"):
            nbr = nbr * int(z[f"tf2/{tag}/nnb"])
        ended = set(z[f"tf2/{tag}/ended"].tolist())
        loaded, end = [], False
        for j in nbr:
            loaded.append(j)
            end = j in ended
            if end:
                break
        out = O.tf2_weights(local, [models[j] for j in loaded], training_end=end)
        for t in range(L):
            ref = z[f"tf2/{tag}/out_{t}"]
            assert out[t].dtype == ref.dtype and np.array_equal(out[t], ref), (tag, t)


def test_closed_form_equals_sequential_in_exact_arithmetic():
    from fractions import Fraction
    alphas = [Fraction(1, 3), Fraction(1, 3), Fraction(2, 7)]
    c = O.closed_form_coeffs(alphas)
    w, xs = Fraction(5), [Fraction(2), Fraction(-1), Fraction(7)]
    seq = w
    for a, x in zip(alphas, xs):
        seq = seq + a * (x - seq)
    assert c[0] * w + sum(cj * x for cj, x in zip(c[1:], xs)) == seq
    assert sum(c) == 1


@pytest.mark.parametrize("variant", ["fast", "4stage_e1", "4stage_e3"])
def test_tf1_cfa_ge_mobilenet_oracle(variant):
    """cfa_ge_2stage_mobilenet.py: vGraph neighbours of the epoch, states re-zeroed per call."""
    z = load_golden("tf1_cfa_ge_mobilenet.npz")
    tag = f"cnn_{variant}"
    K, N, ii, epoch = (int(x) for x in z[f"{tag}/meta"])
    rho, eps, lr1, lr2 = (float(x) for x in z[f"{tag}/hyper"])
    nbr = z[f"{tag}/nbr"].tolist()
    graph = load_golden("topology_mobile.npz")["graph"]
    assert nbr == [kk for kk in range(K) if graph[ii, kk, epoch] == 1]
    local = [z[f"{tag}/local_{t}"] for t in range(4)]
    prev = [[z[f"{tag}/prev{j}_{t}"] for t in range(4)] for j in nbr]
    W = O.tf1_mix(local, prev, eps, [O.tf1_weight_factor(K, ii, j, N - 1) for j in nbr])
    states = [np.zeros(z[f"{tag}/state_out_{t}"].shape) for t in range(4)]
    grads = [[z[f"{tag}/grad{j}_{t}"] for t in range(4)] for j in nbr]
    W = O.tf1_mewma(W, states, grads, rho, lr1, lr2, use_filtered=(variant == "fast"), init=(variant == "4stage_e1"))
    for t in range(4):
        ref = z[f"{tag}/out_{t}"]
        assert np.array_equal(np.asarray(W[t]).reshape(ref.shape), ref), (variant, t)
        assert np.array_equal(states[t], z[f"{tag}/state_out_{t}"]), (variant, "state", t)
