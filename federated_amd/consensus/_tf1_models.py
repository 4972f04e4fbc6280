"""Gradient evaluation of the two TF1 CFA-GE models (not the reduction path).

CFA-GE devices publish, for each neighbour, the gradient of their OWN cost evaluated at that
neighbour's model (cfa_ge_2stage.py:391-433 builds the graph, :512-528 runs one Session per
neighbour). TensorFlow is not part of this stack: the two graphs run as libcfa HIP kernels
(``csrc/cfa_grad.hip``, ``cfa_ge_grad_{cnn,2nn}_rows_f32``), every neighbour model in one
launch with each model's batch split over several workgroups, with TensorFlow's conventions (SAME padding, first-maximum pooling
gradient, relu gradient where the activation is > 0, clip gradient where 1e-15 <= pred <= 0.99).
Inputs are rounded to fp32 as the reference's tf.float32 placeholders round them; gradients
come back as fp32 arrays with the parameter shapes (biases 1-D), like Session.run's outputs.
Without a GPU this raises (no CPU fallback).
"""
from __future__ import annotations

import math
from typing import List, Sequence

import numpy as np
import torch

from ..engine import get_engine


def same_pad(L: int, k: int, s: int):
    """TF SAME padding: out = ceil(L / s), total = max((out - 1) s + k - L, 0), left = total // 2."""
    out = math.ceil(L / s)
    total = max((out - 1) * s + k - L, 0)
    return total // 2, total - total // 2


def _flat(model) -> np.ndarray:
    W1, b1, W2, b2 = model
    return np.concatenate([np.asarray(W1, np.float32).reshape(-1), np.asarray(np.squeeze(b1), np.float32).reshape(-1),
                           np.asarray(W2, np.float32).reshape(-1), np.asarray(np.squeeze(b2), np.float32).reshape(-1)])


def gradients_batched(ml_model: int, x, y, models: Sequence, stride: int = 1, device=None) -> List[list]:
    """Gradients of the device's cost at every model of ``models`` (list of (W1, b1, W2, b2)),
    in ONE kernel launch. x, y and the models are packed into one pinned staging buffer (one
    H2D); the gradients come back with one D2H. Returns one list of four fp32 arrays per model."""
    if not models:
        return []
    from ._runtime import mixer
    hm = mixer() if device is None else None
    eng = hm.engine if hm is not None else get_engine(device)
    W1 = np.asarray(models[0][0])
    shapes = [W1.shape, (int(np.size(models[0][1])),), np.asarray(models[0][2]).shape, (int(np.size(models[0][3])),)]
    sizes = [int(np.prod(s)) for s in shapes]
    P, M = sum(sizes), len(models)
    x = np.asarray(x)
    y = np.asarray(y)
    if x.ndim != 2 or y.ndim != 2 or x.shape[0] != y.shape[0]:
        raise ValueError("x must be [B, inputs] and y [B, classes]")
    nx, ny = x.size, y.size
    B = int(x.shape[0])
    # staging: x, y, the M models, then the int32 row tables of the population-form launch
    # (evaluation m = model m on the one data set), all in one H2D
    total = nx + ny + M * P + 2 * M
    # each evaluation's batch split over several workgroups (partials summed in a fixed order)
    n_ws = int(eng.lib.cfa_ge_grad_workspace_elems(M, B, P))
    if hm is not None:
        st = hm._stream()
        host = hm._cached("h_grad", total, torch.float32, pinned=True)
        dbuf = hm._cached("d_grad", total + M * P, torch.float32)
        h_out = hm._cached("h_grad_out", M * P, torch.float32, pinned=True)
        ws = hm._cached("d_grad_ws", n_ws, torch.float32) if n_ws else None
    else:
        st = torch.cuda.Stream(eng.device)
        host = torch.empty(total, dtype=torch.float32, pin_memory=True)
        dbuf = torch.empty(total + M * P, dtype=torch.float32, device=eng.device)
        h_out = torch.empty(M * P, dtype=torch.float32, pin_memory=True)
        ws = torch.empty(n_ws, dtype=torch.float32, device=eng.device) if n_ws else None
    hv = host.numpy()
    hv[:nx] = x.reshape(-1)            # fp32 rounding, as the tf.float32 placeholders round
    hv[nx:nx + ny] = y.reshape(-1)
    rows = hv[nx + ny + M * P:total].view(np.int32)
    rows[:M] = np.arange(M, dtype=np.int32)
    rows[M:] = 0
    mv = hv[nx + ny:nx + ny + M * P].reshape(M, P)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    for i, m in enumerate(models):
        parts = [np.asarray(m[0]), np.squeeze(m[1]), np.asarray(m[2]), np.squeeze(m[3])]
        for k in range(4):
            if np.size(parts[k]) != sizes[k]:
                raise ValueError("all models must share the first model's shapes")
            mv[i, offs[k]:offs[k + 1]] = np.asarray(parts[k]).reshape(-1)
    with torch.cuda.stream(st):
        dbuf[:total].copy_(host, non_blocking=True)
        xt = dbuf[:nx].view(x.shape)
        yt = dbuf[nx:nx + ny].view(y.shape)
        mt = dbuf[nx + ny:nx + ny + M * P].view(M, P)
        rt = dbuf[nx + ny + M * P:total].view(torch.int32)
        gt = dbuf[total:total + M * P].view(M, P)
        if ml_model == 1:
            if W1.ndim != 3 or W1.shape[1] != 1:
                raise ValueError("CNN W1 must be [filter, 1, number]")
            geom = {"filter": W1.shape[0], "number": W1.shape[2], "stride": int(stride)}
        elif ml_model == 2:
            geom = {"intermediate_nodes": W1.shape[1]}
        else:
            raise ValueError("Unable to set the ML model paramters")
        eng.grad_rows(ml_model, xt.view(1, *x.shape), yt.view(1, *y.shape), mt, rt[:M], rt[M:], gt, geom,
                      stream=st, workspace=ws)
        h_out.copy_(dbuf[total:total + M * P], non_blocking=True)
        st.synchronize()
        g = h_out.numpy().reshape(M, P).copy()
    return [[g[i, offs[k]:offs[k + 1]].reshape(shapes[k]) for k in range(4)] for i in range(M)]


def gradients(ml_model: int, x, y, W1, b1, W2, b2, stride: int = 1, device=None) -> list:
    """``gradients_batched`` for one model."""
    return gradients_batched(ml_model, x, y, [(W1, b1, W2, b2)], stride=stride, device=device)[0]
