"""f1 aggregation loops embedded in the reference's drivers (PS_server.py:130-133,
learner_consensus.py:151-152, federated_sample_CNN_CFA_FA.py:86-89 / :130-133 / :280-283).
Fixtures: tests/golden/f1_driver_aggregations.npz, produced by executing those driver lines as
they stand (tests/golden/make_golden.py::case_driver_aggregations).

CPU: the oracle restatement equals the fixtures (dtype, shape, bits).
GPU: federated_amd.server through libcfa equals the fixtures (dtype, shape, bits)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import cfa_oracle as O

KEYS = ("weights1", "biases1", "weights2", "biases2")
L = 6


def _same(a, ref):
    a, ref = np.asarray(a), np.asarray(ref)
    return a.dtype == ref.dtype and a.shape == ref.shape and np.array_equal(a, ref)


def _inputs():
    z = load_golden("f1_driver_aggregations.npz")
    glob_ = [z[f"ps_mqtt/global_{t}"] for t in range(L)]
    D = z["ps_mqtt/storage_0"].shape[0]
    storage = [[z[f"ps_mqtt/storage_{t}"][d] for t in range(L)] for d in range(D)]
    K = z["cfa_fa/c0_weights1"].shape[0]
    c0 = [{k: z[f"cfa_fa/c0_{k}"][d] for k in KEYS} for d in range(K)]
    c1 = [{k: z[f"cfa_fa/c1_{k}"][d] for k in KEYS} for d in range(K)]
    server_file = {k: z[f"cfa_fa/server_file_{k}"] for k in KEYS}
    wval = [z[f"cfa_fa/wval_{k}"] for k in range(4)]
    return z, glob_, storage, c0, c1, server_file, wval


def _zeros():  # federated_sample_CNN_CFA_FA.py:73-76 with filter 16, number 8, multip 21
    return [np.zeros([16, 1, 8]), np.zeros([8]), np.zeros([21 * 8, 8]), np.zeros([8])]


def _check_all(impl):
    z, glob_, storage, c0, c1, server_file, wval = _inputs()
    idx = z["ps_mqtt/idx"]
    for tag in ("a4_u1", "a1_u05", "a6_u1"):
        active, u = z[f"ps_mqtt/{tag}/meta"]
        active = int(active)
        u = 1 if u == 1 else float(u)
        res = impl.ps_mqtt_aggregate([a.copy() for a in glob_], storage, idx, u, active)
        for t in range(L):
            assert _same(res[t], z[f"ps_mqtt/{tag}/out_{t}"]), (tag, t)
    res = impl.learner_consensus_mix([a.copy() for a in glob_], storage[0], 1, 2)
    for t in range(L):
        assert _same(res[t], z[f"learner/out_{t}"]), t
    K = len(c0)
    bal = np.ones(K) * (1 / K)
    srv = impl.cfa_fa_server_init(_zeros(), c0, bal)
    for k in range(4):
        assert _same(srv[k], z[f"cfa_fa/init_{k}"]), ("init", k)
    srv = impl.cfa_fa_server_round(srv, c1, 0.7, bal)
    for k in range(4):
        assert _same(srv[k], z[f"cfa_fa/round_{k}"]), ("round", k)
    cli = impl.cfa_fa_client_mix(*[a.copy() for a in wval], server_file, 0.35)
    for k in range(4):
        assert _same(cli[k], z[f"cfa_fa/client_{k}"]), ("client", k)


def test_oracle_matches_driver_lines():
    _check_all(O)


def test_fixture_records_cited_lines():
    z = load_golden("f1_driver_aggregations.npz")
    assert z["ps_mqtt/src_lines"].tolist() == [130, 133]
    assert z["learner/src_lines"].tolist() == [151, 152]
    assert z["cfa_fa/init_src_lines"].tolist() == [86, 89]
    assert z["cfa_fa/round_src_lines"].tolist() == [130, 133]
    assert z["cfa_fa/client_src_lines"].tolist() == [280, 283]


@pytest.mark.gpu
def test_server_module_identical_to_driver_lines(gpu):
    from federated_amd import server
    _check_all(server)


@pytest.mark.gpu
def test_server_fold_fp32_operands_stay_fp32(gpu):
    """All-fp32 operands with Python-float scalars: numpy keeps the chain in fp32, so does the
    dispatch (fp32 kernels), bit for bit."""
    from federated_amd import server
    rng = np.random.default_rng(3)
    p = [rng.standard_normal(s).astype(np.float32) for s in [(10, 3), (3,)]]
    rx = [rng.standard_normal(s).astype(np.float32) for s in [(10, 3), (3,)]]
    res = server.learner_consensus_mix([a.copy() for a in p], rx, 1, 2)
    ref = O.learner_consensus_mix([a.copy() for a in p], rx, 1, 2)
    for a, r in zip(res, ref):
        assert r.dtype == np.float32 and _same(a, r)
