"""(f3) CFA-GE neighbour-gradient evaluation: the oracle's hand-derived gradients of the two TF1
graphs (cfa_ge_2stage.py:391-433) pinned on the CPU by central finite differences (float64)
and by an independent torch-autograd restatement of the same graphs; the HIP kernels
(cfa_ge_grad_cnn_f32 / cfa_ge_grad_2nn_f32) are checked against the oracle in
tests/test_gpu_grad.py."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import cfa_oracle as orc


# -- independent torch restatement of the TF1 graphs (test infrastructure only) ------------------
def _same_pad(L, k, s):
    out = math.ceil(L / s)
    total = max((out - 1) * s + k - L, 0)
    return total // 2, total - total // 2


def _torch_cost(logits, y):
    pred = torch.softmax(logits, dim=1)
    return torch.mean(-torch.sum(y * torch.log(torch.clamp(pred, 1e-15, 0.99)), dim=1))


def _torch_cnn(x, W1, b1, W2, b2, stride):
    k = W1.shape[0]
    pl, pr = _same_pad(x.shape[1], k, stride)
    h = F.conv1d(F.pad(x.unsqueeze(1), (pl, pr)), W1.permute(2, 1, 0), b1, stride=stride)
    h = torch.relu(h)
    ql, qr = _same_pad(h.shape[2], stride, stride)
    h = F.max_pool1d(F.pad(h, (ql, qr), value=float("-inf")), kernel_size=stride, stride=stride)
    return h.permute(0, 2, 1).reshape(h.shape[0], -1) @ W2 + b2


def _torch_2nn(x, W1, b1, W2, b2):
    return torch.relu(x @ W1 + b1) @ W2 + b2


def _torch_grads(fwd, params, x, y):
    ps = [torch.tensor(p, dtype=torch.float64, requires_grad=True) for p in params]
    loss = _torch_cost(fwd(torch.tensor(x, dtype=torch.float64), *ps), torch.tensor(y, dtype=torch.float64))
    return [g.numpy() for g in torch.autograd.grad(loss, ps)], float(loss.detach())


def _cnn_case(rng, B=6, scale=0.3):
    W1 = rng.standard_normal((16, 1, 8)) * scale
    b1 = rng.standard_normal(8) * 0.1
    W2 = rng.standard_normal((168, 8)) * 0.1
    b2 = rng.standard_normal(8) * 0.1
    x = rng.standard_normal((B, 512))
    y = np.eye(8)[rng.integers(0, 8, B)]
    return [W1, b1, W2, b2], x, y


def test_cnn_oracle_matches_autograd_and_finite_differences():
    rng = np.random.default_rng(1)
    params, x, y = _cnn_case(rng)
    g, cost = orc.tf1_cnn_grads(x, y, *params, stride=5)
    gt, cost_t = _torch_grads(lambda xx, *p: _torch_cnn(xx, *p, stride=5), params, x, y)
    assert abs(cost - cost_t) < 1e-12
    for a, b in zip(g, gt):
        assert a.shape == b.shape and np.max(np.abs(a - b)) <= 1e-12 * max(1.0, np.max(np.abs(b)))
    _fd(lambda p: orc.tf1_cnn_grads(x, y, *p, stride=5)[1], params, g)


def test_2nn_oracle_matches_autograd_and_finite_differences():
    rng = np.random.default_rng(2)
    params = [rng.standard_normal((64, 16)) * 0.2, rng.standard_normal(16) * 0.1,
              rng.standard_normal((16, 8)) * 0.2, rng.standard_normal(8) * 0.1]
    x = rng.standard_normal((5, 64))
    y = np.eye(8)[[1, 2, 3, 4, 0]]
    g, cost = orc.tf1_2nn_grads(x, y, *params)
    gt, cost_t = _torch_grads(_torch_2nn, params, x, y)
    assert abs(cost - cost_t) < 1e-12
    for a, b in zip(g, gt):
        assert np.max(np.abs(a - b)) <= 1e-12 * max(1.0, np.max(np.abs(b)))
    _fd(lambda p: orc.tf1_2nn_grads(x, y, *p)[1], params, g)


def _fd(cost_fn, params, grads, per_param=6, h=1e-6):
    rng = np.random.default_rng(0)
    for k, (p, g) in enumerate(zip(params, grads)):
        for i in rng.choice(p.size, size=min(per_param, p.size), replace=False):
            def f(delta):
                q = [a.copy() for a in params]
                q[k].reshape(-1)[i] += delta
                return cost_fn(q)
            num = (f(h) - f(-h)) / (2 * h)
            assert abs(num - g.reshape(-1)[i]) <= 1e-6 + 1e-5 * abs(num), (k, i, num, g.reshape(-1)[i])


def test_clip_saturation_blocks_the_gradient():
    """Saturated softmax (pred > 0.99): tf.clip_by_value passes no gradient there."""
    rng = np.random.default_rng(3)
    params, x, y = _cnn_case(rng, B=4, scale=3.0)
    params[3] = np.array([40.0, 0, 0, 0, 0, 0, 0, 0])  # class 0 saturates
    y = np.eye(8)[[0, 0, 1, 0]]
    g, _ = orc.tf1_cnn_grads(x, y, *params, stride=5)
    gt, _ = _torch_grads(lambda xx, *p: _torch_cnn(xx, *p, stride=5), params, x, y)
    for a, b in zip(g, gt):
        assert np.allclose(a, b, rtol=1e-10, atol=1e-14)


def test_same_padding_matches_tf_rule():
    # CFA-GE config: 512 inputs, stride 5 -> conv 103 -> pool 21 = multip (federated_sample_CNN_CFA-GE.py:36-42)
    assert _same_pad(512, 16, 5) == (7, 7) and _same_pad(103, 5, 5) == (1, 1)
    logits, pooled, _, _ = orc.tf1_cnn_forward(np.zeros((2, 512)), np.zeros((16, 1, 8)), np.zeros(8),
                                               np.zeros((168, 8)), np.zeros(8), 5)
    assert logits.shape == (2, 8) and pooled.shape == (2, 21, 8)


def test_product_gradients_need_the_gpu():
    """No CPU fallback: without a GPU the f3 entry point raises."""
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from federated_amd.consensus import _tf1_models as M
    rng = np.random.default_rng(4)
    params, x, y = _cnn_case(rng, B=2)
    with pytest.raises(RuntimeError):
        M.gradients(1, x, y, *params, stride=5)
