"""FedAvg parameter server: the oracle against the reference's outputs (CPU),
and the drop-in Parameter_Server classes against the same outputs on the GPU (bit-exact: the
reference is fp32 numpy and libcfa's SEQUENTIAL_DIV rule rounds step for step like it)."""
import os
import random

import numpy as np
import pytest

from conftest import load_golden
from oracle import cfa_oracle as O

L = 6


def _setup(z):
    D = z["models_0"].shape[0]
    models = [[z[f"models_{t}"][d] for t in range(L)] for d in range(D)]
    grads = [[z[f"grads_{t}"][d] for t in range(L)] for d in range(D)]
    glob_ = [z[f"global_{t}"] for t in range(L)]
    return D, models, grads, glob_


def _expected_sources(z, tag, D):
    agg, active, epoch = (int(x) for x in z[f"{tag}/meta"])
    if tag.startswith("ps2"):
        return [int(k) for k in z["indexes_tx"][:, epoch]]
    random.seed(5)
    return random.sample(range(D), active)


def test_ps_oracle_matches_reference():
    z = load_golden("tf2_parameter_server.npz")
    D, models, grads, glob_ = _setup(z)
    for tag in z["cases"]:
        tag = str(tag)
        agg = int(z[f"{tag}/meta"][0])
        if agg == 1:
            continue  # model copy, no arithmetic (tested through the drop-in)
        u = float(z[f"{tag}/u"])
        u = (1 if tag.startswith("ps1") and not tag.startswith("ps1c") else 0.99) if u < 0 else u
        u = 1 if u == 1.0 else u
        src = _expected_sources(z, tag, D)
        pool = grads if "meta" in tag else models
        ended = z[f"{tag}/ended"].tolist()
        if ended:
            first = [k for k in src if k in ended][0]
            out = O.ps_fedavg(glob_, [pool[first]], u, divide=False)
        else:
            out = O.ps_fedavg(glob_, [pool[k] for k in src], u)
        for t in range(L):
            assert np.array_equal(out[t], z[f"{tag}/out_{t}"]), (tag, t)


def _obj(layers):
    a = np.empty(len(layers), dtype=object)
    for i, l in enumerate(layers):
        a[i] = l
    return a


@pytest.mark.gpu
def test_ps_dropin_bitexact(tmp_path, monkeypatch):
    from federated_amd.consensus import parameter_server, parameter_server_099, parameter_server_v2
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("FEDERATED_AMD_PAUSE_SCALE", "0")
    os.makedirs("results")
    z = load_golden("tf2_parameter_server.npz")
    D, models, grads, glob_ = _setup(z)
    for tag in z["cases"]:
        tag = str(tag)
        agg, active, epoch = (int(x) for x in z[f"{tag}/meta"])
        u = float(z[f"{tag}/u"])
        ended = set(z[f"{tag}/ended"].tolist())
        for k in range(D):
            np.save(f"results/dump_train_model{k}.npy", _obj(models[k]), allow_pickle=True)
            np.save(f"results/dump_train_grad{k}.npy", _obj(grads[k]), allow_pickle=True)
            np.savez(f"results/dump_train_variables{k}.npz", epoch_count=10, training_end=k in ended,
                     loss=z["losses"][k])
        params = _obj([a.copy() for a in glob_])
        kw = {} if u < 0 else {"update_factor": (1 if u == 1.0 else u)}
        if tag.startswith("ps2"):
            p = parameter_server_v2.Parameter_Server(D, params, active, z["indexes_tx"], **kw)
        elif tag.startswith("ps1c"):
            p = parameter_server_099.Parameter_Server(D, params, active, **kw)
        else:
            p = parameter_server.Parameter_Server(D, params, active, **kw)
        random.seed(5)
        res = p.federated_metalearning(epoch, agg) if "meta" in tag else p.federated_target_weights_aggregation(epoch, agg)
        probe = random.random()
        for t in range(L):
            assert np.array_equal(np.asarray(res[t]), z[f"{tag}/out_{t}"]), (tag, t)
        assert probe == float(z[f"{tag}/rng_probe"]), tag
