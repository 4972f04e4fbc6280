"""Randomised differential check of the CPU oracle against the reference's own consensus modules.

The golden fixtures (tests/golden/*.npz) pin the oracle on fixed cases. This test runs the
reference's modules themselves (from /root/reference, with the TF stubs and the temporary working
directory of tests/golden/make_golden.py; nothing is copied into the repo) on seeded random cases
the fixtures do not hold: device counts, neighbour counts, eps values, layer shapes, neighbour
lists and training_end flags, and requires the oracle to reproduce every output bit for bit.

- TF1 cfa.py (a1, TF1/consensus/cfa.py:35-154): k-regular neighbours, epoch-0 publish then an
  epoch-1 mix, fp64 results under numpy 2 (and the reference's UnboundLocalError for a device
  left without a neighbour, which the drop-ins reproduce: test_tf1_no_neighbour.py);
- TF2 consensus_v3 weights (a5, consensus_v3.py:73-159) with the eps override and the
  training_end transfer, and consensus_v4 gradients (a6, consensus_v4.py:219-260) with the
  caller's eps.

The reference tree exists only in the build container, so the test is skipped elsewhere (the GPU
box): it checks the checker, the GPU tests then compare the kernels with the oracle.
"""
import importlib.util
import os
import sys

import numpy as np
import pytest

from oracle import cfa_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("cfa_make_golden", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)

pytestmark = pytest.mark.skipif(not os.path.isdir(MG.TF1), reason="reference tree not present (build container only)")

_STUBBED = ("tensorflow", "tensorflow.keras", "tensorflow.keras.layers", "tensorflow.keras.models", "keras",
            "keras.utils")


@pytest.fixture(scope="module")
def ref():
    saved = {k: sys.modules.get(k) for k in _STUBBED}
    MG.install_stubs()
    try:
        yield {
            "cfa": MG.load_ref(os.path.join(MG.TF1, "consensus", "cfa.py"), "fuzz_ref_cfa"),
            "v3": MG.load_ref(os.path.join(MG.TF2, "MNIST_dataset", "consensus", "consensus_v3.py"), "fuzz_ref_v3"),
            "v4": MG.load_ref(os.path.join(MG.TF2, "MNIST_dataset", "consensus", "consensus_v4.py"), "fuzz_ref_v4"),
        }
    finally:
        for k, v in saved.items():  # the stubs must not leak into the rest of the session
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def _shapes(rng):
    a, b, c = (int(x) for x in rng.integers(1, 48, size=3))
    return [(a, b), (b,), (b, c), (c,)]


@pytest.mark.parametrize("seed", range(8))
def test_tf1_cfa_random_configs(ref, seed):
    rng = np.random.default_rng(9100 + seed)
    K = int(rng.integers(3, 10))
    N = int(rng.integers(1, min(5, K)))
    eps = float(rng.uniform(0.05, 1.0))
    shapes = _shapes(rng)
    scale = float(rng.choice([1e-3, 1.0, 30.0]))
    e0 = [MG.gen_model(rng, shapes, scale) for _ in range(K)]
    e1 = [MG.gen_model(rng, shapes, scale) for _ in range(K)]
    with MG.Workdir():
        procs = [ref["cfa"].CFA_process(True, K, j, N) for j in range(K)]
        for j in range(K):
            W1, b1, W2, b2 = e0[j]
            procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps)
        for ii in range(K):
            W1, b1, W2, b2 = e1[ii]
            nbr = O.tf1_kregular(ii, N, K)
            assert nbr.tolist() == np.asarray(procs[ii].neighbor_vec).tolist(), (K, N, ii)
            if nbr.size == 0:  # N = 1 leaves interior devices without a neighbour: the reference
                with pytest.raises(UnboundLocalError):  # fails (test_tf1_no_neighbour.py: so do the drop-ins)
                    procs[ii].getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), eps)
                continue
            res = procs[ii].getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), eps)
            wf = [O.tf1_weight_factor(K, ii, int(j), N - 1) for j in nbr]
            got = O.tf1_mix(e1[ii], [e0[int(j)] for j in nbr], eps, wf)
            for t in range(4):
                want = np.asarray(res[t])
                assert got[t].dtype == want.dtype, (K, N, ii, t)
                assert np.array_equal(np.asarray(got[t]).reshape(want.shape), want), (K, N, ii, t)


@pytest.mark.parametrize("seed", range(8))
def test_tf2_v3_weights_and_v4_grads_random_configs(ref, seed):
    rng = np.random.default_rng(9200 + seed)
    D = int(rng.integers(4, 11))
    n = int(rng.integers(1, min(6, D)))
    shapes = [(int(x),) if i % 2 else (int(x), int(y)) for i, (x, y) in enumerate(rng.integers(1, 40, size=(4, 2)))]
    models = [MG.gen_model(rng, shapes) for _ in range(D)]
    grads = [MG.gen_model(rng, shapes, 0.1) for _ in range(D)]
    local = MG.gen_model(rng, shapes)
    local_g = MG.gen_model(rng, shapes, 0.1)
    nbr = [int(j) for j in rng.choice(np.arange(1, D), size=n, replace=False)]
    ended = {int(rng.choice(nbr))} if rng.random() < 0.4 else set()
    eps = float(rng.uniform(0.05, 0.95))
    with MG.Workdir():
        for k in range(D):
            MG.publish_tf2(k, models[k], 10, k in ended, grads[k])
        p3 = ref["v3"].CFA_process(D, 0, 2)
        loc = MG.obj_array([a.copy() for a in local])
        p3.update_local_model(loc)
        res_w = p3.federated_weights_computing(nbr, n, 10, eps, 0, 30)
        p4 = ref["v4"].CFA_process(D, 0, 2)
        p4.update_local_model(MG.obj_array([a.copy() for a in local]))
        gl = MG.obj_array([a.copy() for a in local_g])
        p4.update_local_gradient(gl)
        # consensus_v4.py:225-246: one neighbour is passed as a scalar id (the ring rule's form)
        res_g = p4.federated_grads_computing(nbr if n > 1 else nbr[0], n, 10, eps, 1)
    # both stop loading at the first neighbour that reports training_end (v3 :139-141, v4 :233-235)
    upto = next((i + 1 for i, j in enumerate(nbr) if j in ended), len(nbr))
    want_w = O.tf2_weights(local, [models[j] for j in nbr[:upto]], training_end=bool(ended))
    for t in range(len(shapes)):
        assert np.array_equal(np.asarray(res_w[t]), want_w[t]), (D, n, sorted(ended), t)
    want_g = O.tf2_grads_v4(local_g, [grads[j] for j in nbr[:upto]], eps)
    for t in range(len(shapes)):
        assert np.array_equal(np.asarray(res_g[t]), want_g[t]), (D, n, t)


@pytest.mark.parametrize("fast", [True, False])
def test_tf1_cfa_ge_without_neighbour_raises_in_the_reference(ref, fast):
    """The case test_tf1_no_neighbour.py pins for the drop-in: the reference's CFA-GE negotiation
    (cfa_ge_2stage.py:388-470 fast, :129-211 4-stage) fails with UnboundLocalError when the
    device has no neighbour (N = 1, interior device), before it publishes its epoch-1 model."""
    ge = MG.load_ref(os.path.join(MG.TF1, "consensus", "cfa_ge_2stage.py"), "fuzz_ref_cfa_ge")
    rng = np.random.default_rng(9300 + int(fast))
    K, ii, epoch = 5, 2, 1
    with MG.Workdir():
        p = ge.CFA_ge_process(True, K, ii, 1, 0.99)
        p.setCNNparameters(16, 8, 5, 5, 21, 8, 512)
        assert np.asarray(p.get_connectivity(ii, 1, K)).size == 0
        W1, b1, W2, b2 = MG.gen_model(rng, MG.SHAPES_CNN_GE)
        st = [np.zeros(tuple(s) + (1,)) for s in MG.SHAPES_CNN_GE]
        fn = p.getFederatedWeight_gradients_fast if fast else p.getFederatedWeight_gradients
        with pytest.raises(UnboundLocalError):
            fn(W1, W2, b1, b2, epoch, np.zeros(3), 0, None, None, st[0], st[2], st[1], st[3], 1.0, 0.1, 0.05)
        assert not os.path.isfile(f"datamat{ii}_{epoch}.mat")


@pytest.mark.parametrize("seed", range(10))
def test_tf1_ongraphs_mode1_random_configs(ref, seed):
    """cfa_ongraphs.py:152-314, consensus mode 1 with the caller's neighbour list (graph != 0):
    random device, neighbour list, eps and compression mode on models in the regime the
    compression thresholds act on; the oracle's fp64 chain, epilogue and counter_param match."""
    og = MG.load_ref(os.path.join(MG.TF1, "consensus", "cfa_ongraphs.py"), "fuzz_ref_ongraphs")
    rng = np.random.default_rng(9400 + seed)
    K = 5  # the vGraph.mat fixture's device count
    ii = int(rng.integers(0, K))
    others = [j for j in range(K) if j != ii]
    nb = [int(j) for j in rng.choice(others, size=int(rng.integers(1, K)), replace=False)]
    eps = float(rng.uniform(0.1, 1.0))
    comp = int(rng.integers(0, 5))
    m0 = MG.ongraphs_models(rng, K, MG.SHAPES_ONGRAPHS_SMALL)
    m1 = MG.ongraphs_models(rng, K, MG.SHAPES_ONGRAPHS_SMALL)
    with MG.Workdir():
        procs = [og.CFA_process(True, K, j, 2, 6, comp, 1) for j in range(K)]
        for j in range(K):
            W1, b1, W2, b2 = m0[j]
            procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps, [], False)
        W1, b1, W2, b2 = [a.copy() for a in m1[ii]]
        res = procs[ii].getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), eps, nb, False)
    local = [a.copy() for a in m1[ii]]
    wf = [O.tf1_weight_factor(K, ii, j, len(nb)) for j in nb]
    out = O.tf1_mix(local, [m0[j] for j in nb], eps, wf)
    counter = O.tf1_compress(out[2], local[2], comp)
    for t in range(4):
        want = np.asarray(res[t])
        assert np.array_equal(np.asarray(out[t]).reshape(want.shape), want), (ii, nb, comp, t)
    assert counter == int(res[4]), (ii, nb, comp)


@pytest.mark.parametrize("seed", range(8))
def test_parameter_server_v2_random_configs(ref, seed):
    """parameter_server_v2.py:83-164 FedAvg: the active devices of column ``epoch`` of indexes_tx,
    p <- p + u (x_k - p) / C in order, or the transfer from the first device reporting
    training_end (:150-157); random device counts, active sets, update factors and ended flags."""
    ps2 = MG.load_ref(os.path.join(MG.TF2, "MNIST_dataset", "consensus", "parameter_server_v2.py"), "fuzz_ref_ps2")
    rng = np.random.default_rng(9500 + seed)
    D = int(rng.integers(3, 10))
    active = int(rng.integers(1, D + 1))
    epochs = 4
    indexes_tx = np.stack([rng.permutation(D)[:active] for _ in range(epochs)], axis=1)
    epoch = int(rng.integers(0, epochs))
    u = float(rng.uniform(0.5, 1.0))
    shapes = [(int(x),) if i % 2 else (int(x), int(y)) for i, (x, y) in enumerate(rng.integers(1, 30, size=(4, 2)))]
    models = [MG.gen_model(rng, shapes) for _ in range(D)]
    glob_ = MG.gen_model(rng, shapes)
    chosen = [int(k) for k in indexes_tx[:, epoch]]
    ended = {int(rng.choice(chosen))} if rng.random() < 0.3 else set()
    with MG.Workdir():
        for k in range(D):
            MG.publish_tf2(k, models[k], 10, k in ended)
        p = ps2.Parameter_Server(D, MG.obj_array([a.copy() for a in glob_]), active, indexes_tx, update_factor=u)
        res = p.federated_target_weights_aggregation(epoch, 0)
    if ended:
        first = next(k for k in chosen if k in ended)
        want = O.ps_fedavg(glob_, [models[first]], u, divide=False)
    else:
        want = O.ps_fedavg(glob_, [models[k] for k in chosen], u)
    for t in range(len(shapes)):
        assert np.array_equal(np.asarray(res[t]), want[t]), (D, active, epoch, sorted(ended), t)


@pytest.mark.parametrize("seed", range(6))
def test_cfa_ge_random_configs(ref, seed):
    """cfa_ge_2stage.py: the fast negotiation (:388-635) and the 4-stage one (:129-385, epoch 1
    initialises the states, later epochs filter them): stage-1 mix with the previous epoch's
    models, then the MEWMA / SGD update from the neighbours' gradient slots, random K, N, rho,
    eps and learning rates, CNN geometry of federated_sample_CNN_CFA-GE.py:36-42."""
    ge = MG.load_ref(os.path.join(MG.TF1, "consensus", "cfa_ge_2stage.py"), f"fuzz_ref_cfa_ge_{seed}")
    rng = np.random.default_rng(9600 + seed)
    variant = ("fast", "4stage_e1", "4stage_e3")[seed % 3]
    K = int(rng.integers(4, 10))
    N = int(rng.integers(2, min(5, K)))
    ii = int(rng.integers(0, K))
    rho, eps = float(rng.uniform(0.5, 0.999)), float(rng.uniform(0.2, 1.0))
    lr1, lr2 = float(rng.uniform(0.01, 0.2)), float(rng.uniform(0.01, 0.2))
    epoch = {"fast": int(rng.integers(1, 6)), "4stage_e1": 1, "4stage_e3": 3}[variant]
    shapes = MG.SHAPES_CNN_GE
    prev = [MG.gen_model(rng, shapes) for _ in range(K)]
    cur = [MG.gen_model(rng, shapes) for _ in range(K)]
    grads = [[rng.standard_normal(tuple(s) + (K,)) for s in shapes] for _ in range(K)]
    local = MG.gen_model(rng, shapes)
    states = [rng.standard_normal(tuple(s) + (N,)) for s in shapes]
    grad_epoch = epoch - 1 if variant == "fast" else epoch
    with MG.Workdir():
        p = ge.CFA_ge_process(True, K, ii, N, rho)
        p.setCNNparameters(16, 8, 5, 5, 21, 8, 512)
        nbr = np.asarray(p.get_connectivity(ii, N, K))
        for j in range(K):
            W1, b1, W2, b2 = prev[j]
            MG.sio.savemat(f"datamat{j}_{epoch - 1}.mat", {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
            if variant != "fast" and j != ii:
                W1, b1, W2, b2 = cur[j]
                MG.sio.savemat(f"datamat{j}_{epoch}.mat", {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
            g = grads[j]
            MG.sio.savemat(f"datagrad{j}_{grad_epoch}.mat", {"grad_weights1": g[0], "grad_biases1": g[1],
                                                            "grad_weights2": g[2], "grad_biases2": g[3],
                                                            "epoch": grad_epoch})
        st = [s.copy() for s in states]
        W1, b1, W2, b2 = local
        fn = p.getFederatedWeight_gradients_fast if variant == "fast" else p.getFederatedWeight_gradients
        res = fn(W1, W2, b1, b2, epoch, np.zeros(3), 0, None, None, st[0], st[2], st[1], st[3], eps, lr1, lr2)
    assert nbr.tolist() == O.tf1_kregular(ii, N, K).tolist()
    wf = [O.tf1_weight_factor(K, ii, int(j), N - 1) for j in nbr]
    W = O.tf1_mix(local, [prev[int(j)] for j in nbr], eps, wf)
    ost = [s.copy() for s in states]
    # the update reads slot ii of each neighbour's [..., devices] gradient (cfa_ge_2stage.py:575-589)
    W = O.tf1_mewma(W, ost, [[g[..., ii] for g in grads[int(j)]] for j in nbr], rho, lr1, lr2,
                    variant == "fast", variant == "4stage_e1")
    for t in range(4):
        want = np.asarray(res[t])
        assert np.array_equal(np.asarray(W[t]).reshape(want.shape), want), (variant, K, N, ii, t)
    for t, r in zip((0, 2, 1, 3), res[4:8]):
        assert np.array_equal(ost[t], np.asarray(r)), (variant, K, N, ii, "state", t)
