"""The TF1 drop-ins fail where the reference fails: a mixing epoch without a neighbour.

The reference's TF1 modules assign their result only inside the neighbour loop, so an epoch with
an empty neighbour list (N = 1 on the k-regular window leaves interior devices without one,
cfa.py:14-32) or a federated process with a single device raises UnboundLocalError
(cfa.py:107-154; cfa_ge_2stage.py:189-211 for the 4-stage negotiation, :449-463 for the fast one).
The drop-ins raise the same error at the same point of the file protocol (cfa.py still publishes
its pre-mix model first, as the reference's savemat precedes the failing line). No GPU work happens
before the error, so these run on the CPU. ``test_oracle_reference_fuzz.py`` checks the reference
itself raises in the same cases.
"""
import os

import numpy as np
import pytest


@pytest.fixture
def workdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("FEDERATED_AMD_PAUSE_SCALE", "0")
    return tmp_path


def _model(rng, shapes):
    return [rng.standard_normal(s).astype(np.float32) for s in shapes]


SHAPES = [(16, 4), (4,), (4, 3), (3,)]


def test_cfa_interior_device_without_neighbour_raises_after_publishing(workdir):
    from federated_amd.consensus.cfa import CFA_process
    rng = np.random.default_rng(1)
    p = CFA_process(True, 5, 2, 1)  # N = 1: interior device 2 has no neighbour (cfa.py:19-24)
    assert p.neighbor_vec.size == 0
    W1, b1, W2, b2 = _model(rng, SHAPES)
    p.getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), 1.0)  # epoch 0 only publishes
    with pytest.raises(UnboundLocalError, match="W_up_l1"):
        p.getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), 1.0)
    assert os.path.isfile("datamat2_1.mat")  # published before the failing line, as the reference


def test_cfa_single_federated_device_raises(workdir):
    from federated_amd.consensus.cfa import CFA_process
    rng = np.random.default_rng(2)
    W1, b1, W2, b2 = _model(rng, SHAPES)
    with pytest.raises(UnboundLocalError, match="W_up_l1"):
        CFA_process(True, 1, 0, 2).getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), 1.0)
    # not federated: the model is published and returned unchanged (cfa.py:147-154)
    out = CFA_process(False, 1, 0, 2).getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), 1.0)
    assert out[0] is W1 and os.path.isfile("datamat0_0.mat")


@pytest.mark.parametrize("fast", [True, False])
def test_cfa_ge_interior_device_without_neighbour_raises(workdir, fast):
    from federated_amd.consensus.cfa_ge_2stage import CFA_ge_process
    rng = np.random.default_rng(3)
    p = CFA_ge_process(True, 5, 2, 1, 0.99)
    W1, b1, W2, b2 = _model(rng, [(16, 1, 8), (8,), (168, 8), (8,)])
    st = [np.zeros(np.shape(a) + (1,)) for a in (W1, W2, b1, b2)]
    fn = p.getFederatedWeight_gradients_fast if fast else p.getFederatedWeight_gradients
    fn(W1, W2, b1, b2, 0, np.zeros(3), None, None, None, *st, 1.0, 0.01, 0.01)  # epoch 0 publishes
    with pytest.raises(UnboundLocalError, match="W_up_l1"):
        fn(W1, W2, b1, b2, 1, np.zeros(3), None, None, None, *st, 1.0, 0.01, 0.01)
    assert not os.path.isfile("datamat2_1.mat")  # the reference fails before publishing epoch 1
