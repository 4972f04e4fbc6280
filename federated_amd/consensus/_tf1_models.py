"""Gradient evaluation of the two TF1 CFA-GE models (not the reduction path).

CFA-GE devices publish, for each neighbour, the gradient of their OWN loss evaluated at that
neighbour's model (cfa_ge_2stage.py:391-433 builds the graph, :512-528 runs it). TensorFlow is
not part of this stack, so the two graphs are restated with torch autograd on the GPU, with
TensorFlow's exact conventions:

* CNN (ML_model 1, :392-405): x[B, input] -> expand to NWC [B, input, 1] -> conv1d(W[filter, 1,
  number], stride, padding='SAME') + b -> relu -> max_pooling1d(pool=stride, stride, 'SAME') ->
  reshape [B, multip*number] (NWC order: position-major, channel-minor) -> softmax(. W2 + b2).
* 2NN (ML_model 2, :407-420): softmax(relu(x W1 + b1) W2 + b2).
* cost = mean_b(-sum_c y * log(clip(pred, 1e-15, 0.99))) (:425-426); gradients w.r.t. the four
  placeholders (:429-430). SAME padding: out = ceil(L / s), total pad = max((out-1)s + k - L, 0),
  left = total // 2 (TF's rule); pooled padding never wins a max.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def _same_pad(L: int, k: int, s: int):
    out = math.ceil(L / s)
    total = max((out - 1) * s + k - L, 0)
    return total // 2, total - total // 2


def _cost(logits, y):
    pred = torch.softmax(logits, dim=1)
    return torch.mean(-torch.sum(y * torch.log(torch.clamp(pred, 1e-15, 0.99)), dim=1))


def cnn_forward(x, W1, b1, W2, b2, stride: int):
    """x [B, L]; W1 [filter, 1, number] (TF WIO); returns logits [B, classes]."""
    k = W1.shape[0]
    xin = x.unsqueeze(1)                          # NCW [B, 1, L]
    pl, pr = _same_pad(x.shape[1], k, stride)
    h = F.conv1d(F.pad(xin, (pl, pr)), W1.permute(2, 1, 0), b1, stride=stride)  # [B, number, L1]
    h = torch.relu(h)
    ql, qr = _same_pad(h.shape[2], stride, stride)
    h = F.max_pool1d(F.pad(h, (ql, qr), value=float("-inf")), kernel_size=stride, stride=stride)
    fc = h.permute(0, 2, 1).reshape(h.shape[0], -1)  # NWC flatten: [B, L2 * number]
    return fc @ W2 + b2


def nn2_forward(x, W1, b1, W2, b2):
    return torch.relu(x @ W1 + b1) @ W2 + b2


def gradients(ml_model: int, x, y, W1, b1, W2, b2, stride: int = 1, device=None):
    """Gradients of the device's cost at the given model, as fp32 numpy arrays with the
    parameter shapes (biases 1-D), like the reference's Session.run outputs."""
    dev = device or (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float32), device=dev)
    params = [t(W1).requires_grad_(), t(np.squeeze(b1)).reshape(-1).requires_grad_(),
              t(W2).requires_grad_(), t(np.squeeze(b2)).reshape(-1).requires_grad_()]
    xx, yy = t(x), t(y)
    if ml_model == 1:
        logits = cnn_forward(xx, *params, stride=stride)
    elif ml_model == 2:
        logits = nn2_forward(xx, *params)
    else:
        raise ValueError("Unable to set the ML model paramters")
    g = torch.autograd.grad(_cost(logits, yy), params)
    return [gi.detach().cpu().numpy() for gi in g]


def gradients_batched(ml_model: int, x, y, models, stride: int = 1, device=None):
    """``gradients`` for several models at once (the CFA-GE neighbour-gradient
    evaluation batched on the GPU): the device's cost at every neighbour model in ONE vectorised
    forward/backward (torch.func.vmap over the stacked parameters). ``models`` = list of
    (W1, b1, W2, b2). Returns one list of four fp32 arrays per model, as ``gradients`` does."""
    from torch.func import grad, vmap
    if not models:
        return []
    dev = device or (torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
    t = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float32), device=dev)
    stack = lambda k, flat: torch.stack([t(np.squeeze(m[k])).reshape(-1) if flat else t(m[k]) for m in models])
    params = (stack(0, False), stack(1, True), stack(2, False), stack(3, True))
    xx, yy = t(x), t(y)
    if ml_model == 1:
        fwd = lambda W1, b1, W2, b2: cnn_forward(xx, W1, b1, W2, b2, stride=stride)
    elif ml_model == 2:
        fwd = lambda W1, b1, W2, b2: nn2_forward(xx, W1, b1, W2, b2)
    else:
        raise ValueError("Unable to set the ML model paramters")
    loss = lambda W1, b1, W2, b2: _cost(fwd(W1, b1, W2, b2), yy)
    g = vmap(grad(loss, argnums=(0, 1, 2, 3)))(*params)
    return [[gk[i].detach().cpu().numpy() for gk in g] for i in range(len(models))]
