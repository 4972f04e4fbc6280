"""Randomised parity of the drop-in consensus classes (HIP kernels) with the oracle.

The golden replays (test_gpu_consensus_golden.py) run the reference's fixed scenarios; this runs
the same drop-in classes through the same file protocol on seeded random configurations (device
and neighbour counts, eps, odd layer shapes, value scales, compression modes, training_end
flags, parameter-server active sets), checked bit for bit against the oracle, which
tests/test_oracle_reference_fuzz.py pins to the reference on the same kind of random cases:

- TF1 cfa.py (fp64 results under numpy 2; cfa.py:35-154);
- cfa_ongraphs.py consensus mode 1 with the compression epilogue and counter_param (:152-314);
- TF2 consensus_v3 weights (eps override, training_end transfer; consensus_v3.py:73-159) and
  consensus_v4 gradients (caller's eps; consensus_v4.py:219-260);
- parameter_server_v2 FedAvg (parameter_server_v2.py:83-164).
"""
import os

import numpy as np
import pytest

from oracle import cfa_oracle as O

pytestmark = pytest.mark.gpu

# CFA_DROPIN_FUZZ_CASES (default 6) seeds per drop-in class; CFA_DROPIN_FUZZ_SEED shifts them
SEEDS = [int(os.environ.get("CFA_DROPIN_FUZZ_SEED", "0")) + k
         for k in range(int(os.environ.get("CFA_DROPIN_FUZZ_CASES", "6")))]


@pytest.fixture
def workdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("FEDERATED_AMD_PAUSE_SCALE", "0")
    os.makedirs("results")
    return tmp_path


def _f32(rng, shape, scale=1.0):
    return (rng.standard_normal(shape) * scale).astype(np.float32)


def _model(rng, shapes, scale=1.0):
    return [_f32(rng, s, scale) for s in shapes]


def _obj(layers):
    a = np.empty(len(layers), dtype=object)
    for i, l in enumerate(layers):
        a[i] = l
    return a


def _same(got, want):
    got = np.asarray(got)
    return got.dtype == want.dtype and np.array_equal(got.reshape(want.shape), want)


@pytest.mark.parametrize("seed", SEEDS)
def test_tf1_cfa_dropin_random(workdir, seed):
    from federated_amd.consensus.cfa import CFA_process
    rng = np.random.default_rng(9700 + seed)
    K = int(rng.integers(3, 10))
    N = int(rng.integers(2, min(5, K)))
    eps = float(rng.uniform(0.05, 1.0))
    a, b, c = (int(x) for x in rng.integers(1, 200, size=3))
    shapes = [(a, b), (b,), (b, c), (c,)]
    scale = float(rng.choice([1e-3, 1.0, 30.0]))
    e0 = [_model(rng, shapes, scale) for _ in range(K)]
    e1 = [_model(rng, shapes, scale) for _ in range(K)]
    procs = [CFA_process(True, K, j, N) for j in range(K)]
    for j in range(K):
        W1, b1, W2, b2 = e0[j]
        procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps)
    for ii in range(K):
        nbr = O.tf1_kregular(ii, N, K)
        W1, b1, W2, b2 = e1[ii]
        res = procs[ii].getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), eps)
        wf = [O.tf1_weight_factor(K, ii, int(j), N - 1) for j in nbr]
        want = O.tf1_mix(e1[ii], [e0[int(j)] for j in nbr], eps, wf)
        want = [want[0], np.squeeze(want[1]), want[2], np.squeeze(want[3])]
        for t in range(4):
            assert _same(res[t], np.asarray(want[t])), (K, N, ii, t)


@pytest.mark.parametrize("seed", SEEDS)
def test_tf1_ongraphs_mode1_dropin_random(workdir, seed):
    from federated_amd.consensus.cfa_ongraphs import CFA_process
    rng = np.random.default_rng(9800 + seed)
    K = int(rng.integers(3, 9))
    ii = int(rng.integers(0, K))
    nb = [int(j) for j in rng.choice([j for j in range(K) if j != ii], size=int(rng.integers(1, K)), replace=False)]
    eps = float(rng.uniform(0.1, 1.0))
    comp = int(rng.integers(0, 5))
    w2 = (int(rng.integers(1, 700)), 6)
    shapes = [(3, 3, 1, 4), (4,), w2, (6,)]
    base = _f32(rng, w2, 0.01)  # the regime the compression thresholds act on (W2 near zero, close models)

    def model():
        m = _model(rng, shapes)
        m[2] = (base + _f32(rng, w2, 3e-4)).astype(np.float32)
        return m
    m0 = [model() for _ in range(K)]
    m1 = [model() for _ in range(K)]
    procs = [CFA_process(True, K, j, 2, 6, comp, 1) for j in range(K)]
    for j in range(K):
        W1, b1, W2, b2 = m0[j]
        procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps, [], False)
    W1, b1, W2, b2 = [x.copy() for x in m1[ii]]
    res = procs[ii].getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), eps, nb, False)
    wf = [O.tf1_weight_factor(K, ii, j, len(nb)) for j in nb]
    want = O.tf1_mix([x.copy() for x in m1[ii]], [m0[j] for j in nb], eps, wf)
    counter = O.tf1_compress(want[2], m1[ii][2], comp)
    for t in range(4):
        assert np.array_equal(np.asarray(res[t]).reshape(np.shape(want[t])), want[t]), (K, ii, nb, comp, t)
    assert res[4] == counter, (K, ii, nb, comp)


@pytest.mark.parametrize("seed", SEEDS)
def test_tf2_dropin_random(workdir, seed):
    from federated_amd.consensus import consensus_v3, consensus_v4
    rng = np.random.default_rng(9900 + seed)
    D = int(rng.integers(4, 11))
    n = int(rng.integers(1, min(6, D)))
    shapes = [(int(x),) if i % 2 else (int(x), int(y))
              for i, (x, y) in enumerate(rng.integers(1, 300, size=(int(rng.integers(2, 7)), 2)))]
    models = [_model(rng, shapes) for _ in range(D)]
    grads = [_model(rng, shapes, 0.1) for _ in range(D)]
    local, local_g = _model(rng, shapes), _model(rng, shapes, 0.1)
    nbr = [int(j) for j in rng.choice(np.arange(1, D), size=n, replace=False)]
    ended = {int(rng.choice(nbr))} if rng.random() < 0.4 else set()
    eps = float(rng.uniform(0.05, 0.95))
    for k in range(D):
        np.save(f"results/dump_train_model{k}.npy", _obj(models[k]), allow_pickle=True)
        np.save(f"results/dump_train_grad{k}.npy", _obj(grads[k]), allow_pickle=True)
        np.savez(f"results/dump_train_variables{k}.npz", frame_count=10, epoch_count=10, training_end=k in ended,
                 loss=0.5)
    p3 = consensus_v3.CFA_process(D, 0, 2)
    loc = _obj([x.copy() for x in local])
    p3.update_local_model(loc)
    res_w = p3.federated_weights_computing(nbr, n, 10, eps, 0, 30)
    p4 = consensus_v4.CFA_process(D, 0, 2)
    p4.update_local_model(_obj([x.copy() for x in local]))
    gl = _obj([x.copy() for x in local_g])
    p4.update_local_gradient(gl)
    res_g = p4.federated_grads_computing(nbr if n > 1 else nbr[0], n, 10, eps, 1)
    upto = next((i + 1 for i, j in enumerate(nbr) if j in ended), len(nbr))
    want_w = O.tf2_weights(local, [models[j] for j in nbr[:upto]], training_end=bool(ended))
    want_g = O.tf2_grads_v4(local_g, [grads[j] for j in nbr[:upto]], eps)
    for t in range(len(shapes)):
        assert _same(res_w[t], want_w[t]), (D, n, sorted(ended), t)
        assert _same(loc[t], want_w[t]), (D, n, "in place", t)
        assert _same(res_g[t], want_g[t]), (D, n, "grads", t)


@pytest.mark.parametrize("seed", SEEDS)
def test_parameter_server_v2_dropin_random(workdir, seed):
    from federated_amd.consensus import parameter_server_v2
    rng = np.random.default_rng(10000 + seed)
    D = int(rng.integers(3, 10))
    active = int(rng.integers(1, D + 1))
    indexes_tx = np.stack([rng.permutation(D)[:active] for _ in range(4)], axis=1)
    epoch = int(rng.integers(0, 4))
    u = float(rng.uniform(0.5, 1.0))
    shapes = [(int(x),) if i % 2 else (int(x), int(y)) for i, (x, y) in enumerate(rng.integers(1, 300, size=(4, 2)))]
    models = [_model(rng, shapes) for _ in range(D)]
    glob_ = _model(rng, shapes)
    chosen = [int(k) for k in indexes_tx[:, epoch]]
    ended = {int(rng.choice(chosen))} if rng.random() < 0.3 else set()
    for k in range(D):
        np.save(f"results/dump_train_model{k}.npy", _obj(models[k]), allow_pickle=True)
        np.savez(f"results/dump_train_variables{k}.npz", frame_count=10, epoch_count=10, training_end=k in ended,
                 loss=0.5)
    p = parameter_server_v2.Parameter_Server(D, _obj([x.copy() for x in glob_]), active, indexes_tx, update_factor=u)
    res = p.federated_target_weights_aggregation(epoch, 0)
    if ended:
        first = next(k for k in chosen if k in ended)
        want = O.ps_fedavg(glob_, [models[first]], u, divide=False)
    else:
        want = O.ps_fedavg(glob_, [models[k] for k in chosen], u)
    for t in range(len(shapes)):
        assert _same(res[t], np.asarray(want[t])), (D, active, epoch, sorted(ended), t)
