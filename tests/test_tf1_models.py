"""The torch restatement of the two TF1 CFA-GE graphs (off the reduction path):
autograd gradients against central finite differences in float64, on CPU."""
import numpy as np
import pytest
import torch

from federated_amd.consensus import _tf1_models as M


def _fd_check(forward, params, x, y, idx_per_param=6, h=1e-6):
    ps = [torch.tensor(p, dtype=torch.float64, requires_grad=True) for p in params]
    xx, yy = torch.tensor(x, dtype=torch.float64), torch.tensor(y, dtype=torch.float64)
    loss = M._cost(forward(xx, *ps), yy)
    grads = torch.autograd.grad(loss, ps)
    rng = np.random.default_rng(0)
    for p, g in zip(ps, grads):
        flat = p.detach().reshape(-1)
        for i in rng.choice(flat.numel(), size=min(idx_per_param, flat.numel()), replace=False):
            def f(delta):
                q = [t.detach().clone() for t in ps]
                k = [j for j, t in enumerate(ps) if t is p][0]
                q[k].reshape(-1)[i] += delta
                return float(M._cost(forward(xx, *q), yy))
            num = (f(h) - f(-h)) / (2 * h)
            assert abs(num - float(g.reshape(-1)[i])) <= 1e-5 + 1e-4 * abs(num), (i, num, float(g.reshape(-1)[i]))


def test_cnn_gradients_finite_differences():
    rng = np.random.default_rng(1)
    # federated_sample_CNN_CFA-GE.py:36-42 shapes, small weights so softmax is not clipped
    W1 = rng.standard_normal((16, 1, 8)) * 0.1
    b1 = rng.standard_normal(8) * 0.1
    W2 = rng.standard_normal((168, 8)) * 0.05
    b2 = rng.standard_normal(8) * 0.05
    x = rng.standard_normal((4, 512))
    y = np.eye(8)[[0, 3, 5, 7]]
    _fd_check(lambda xx, *p: M.cnn_forward(xx, *p, stride=5), [W1, b1, W2, b2], x, y)
    g = M.gradients(1, x, y, W1, b1, W2, b2, stride=5, device=torch.device("cpu"))
    assert [a.shape for a in g] == [(16, 1, 8), (8,), (168, 8), (8,)]


def test_2nn_gradients_finite_differences():
    rng = np.random.default_rng(2)
    W1, b1 = rng.standard_normal((64, 16)) * 0.2, rng.standard_normal(16) * 0.1
    W2, b2 = rng.standard_normal((16, 8)) * 0.2, rng.standard_normal(8) * 0.1
    x = rng.standard_normal((5, 64))
    y = np.eye(8)[[1, 2, 3, 4, 0]]
    _fd_check(M.nn2_forward, [W1, b1, W2, b2], x, y)


def test_same_padding_shapes_match_tf_rule():
    # FL_CFA_CNN_tf2/CFA-GE config: 512 inputs, stride 5 -> conv 103 -> pool 21 = multip
    x = torch.zeros(2, 512)
    out = M.cnn_forward(x, torch.zeros(16, 1, 8), torch.zeros(8), torch.zeros(168, 8), torch.zeros(8), stride=5)
    assert out.shape == (2, 8)
    assert M._same_pad(512, 16, 5) == (7, 7) and M._same_pad(103, 5, 5) == (1, 1)


@pytest.mark.parametrize("ml", [1, 2])
def test_batched_gradients_match_per_model(ml):
    """gradients_batched (all neighbour models in one vmapped forward/backward, f3) equals the
    per-model evaluation within fp32 tolerance (1e-5 normwise per tensor)."""
    import torch
    from conftest import normwise_close
    from federated_amd.consensus import _tf1_models as M
    rng = np.random.default_rng(ml)
    if ml == 1:
        shapes, xdim, stride = [(16, 1, 8), (8,), (168, 8), (8,)], 512, 5
    else:
        shapes, xdim, stride = [(64, 16), (16,), (16, 8), (8,)], 64, 1
    models = [[(rng.standard_normal(s) * 0.1).astype(np.float32) for s in shapes] for _ in range(4)]
    x = rng.standard_normal((6, xdim)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[np.arange(6) % 8]
    cpu = torch.device("cpu")
    batched = M.gradients_batched(ml, x, y, models, stride=stride, device=cpu)
    assert M.gradients_batched(ml, x, y, [], stride=stride, device=cpu) == []
    for m, gb in zip(models, batched):
        for a, r in zip(gb, M.gradients(ml, x, y, *m, stride=stride, device=cpu)):
            assert a.shape == r.shape and normwise_close(a, r)
