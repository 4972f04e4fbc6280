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

_STREAMS: dict = {}


def same_pad(L: int, k: int, s: int):
    """TF SAME padding: out = ceil(L / s), total = max((out - 1) s + k - L, 0), left = total // 2."""
    out = math.ceil(L / s)
    total = max((out - 1) * s + k - L, 0)
    return total // 2, total - total // 2


def _flat(model) -> np.ndarray:
    W1, b1, W2, b2 = model
    return np.concatenate([np.asarray(W1, np.float32).reshape(-1), np.asarray(np.squeeze(b1), np.float32).reshape(-1),
                           np.asarray(W2, np.float32).reshape(-1), np.asarray(np.squeeze(b2), np.float32).reshape(-1)])


class _GradPlan:
    """Reusable state of one gradient-evaluation shape on one thread: pinned staging (x, y, the
    M models, the int32 row tables), its device copy, the batch-split workspace and a pinned
    output that the kernel writes directly (zero-copy), plus the bound launch arguments."""

    def __init__(self, eng, ml_model, shapes, M, x_shape, y_shape, geom):
        self.eng, self.lib = eng, eng.lib
        self.shapes = shapes
        self.sizes = [int(np.prod(sh)) for sh in shapes]
        self.offs = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        P = self.P = int(self.offs[-1])
        self.M = M
        nx, ny = int(np.prod(x_shape)), int(np.prod(y_shape))
        self.nx, self.ny = nx, ny
        total = self.total = nx + ny + M * P + 2 * M
        self.host = torch.empty(total, dtype=torch.float32, pin_memory=True)
        self.out = torch.empty(M * P, dtype=torch.float32, pin_memory=True)
        self.dev = torch.empty(total, dtype=torch.float32, device=eng.device)
        B = int(x_shape[0])
        n_ws = int(self.lib.cfa_ge_grad_workspace_elems(M, B, P))
        self.ws = torch.empty(max(n_ws, 1), dtype=torch.float32, device=eng.device)
        hv = self.host.numpy()
        self.xv, self.yv = hv[:nx].reshape(x_shape), hv[nx:nx + ny].reshape(y_shape)
        self.mv = hv[nx + ny:nx + ny + M * P].reshape(M, P)
        self.views = [[self.mv[i, self.offs[k]:self.offs[k + 1]] for k in range(4)] for i in range(M)]
        rows = hv[nx + ny + M * P:total].view(np.int32)
        rows[:M] = np.arange(M, dtype=np.int32)
        rows[M:] = 0
        d = self.dev.data_ptr()
        out = eng.host_device_ptr(self.out)
        xp, yp, mp = d, d + 4 * nx, d + 4 * (nx + ny)
        rp = d + 4 * (nx + ny + M * P)
        common = (self.ws.data_ptr(), n_ws, M)
        if ml_model == 1:
            self.fn = self.lib.cfa_ge_grad_cnn_rows_f32
            self.args = (xp, yp, B, int(x_shape[1]), int(y_shape[1]), int(geom["filter"]), int(geom["number"]),
                         int(geom["stride"]), mp, rp, rp + 4 * M, out) + common
            self.name = "cfa_ge_grad_cnn_rows_f32"
        else:
            self.fn = self.lib.cfa_ge_grad_2nn_rows_f32
            self.args = (xp, yp, B, int(x_shape[1]), int(geom["intermediate_nodes"]), int(y_shape[1]), mp, rp,
                         rp + 4 * M, out) + common
            self.name = "cfa_ge_grad_2nn_rows_f32"
        self.host_ptr, self.dev_ptr = self.host.data_ptr(), d
        self._sh = None

    def run(self, x, y, models, st) -> List[list]:
        np.copyto(self.xv, x, casting="unsafe")  # fp32 rounding, as the tf.float32 placeholders round
        np.copyto(self.yv, y, casting="unsafe")
        sizes = self.sizes
        for i, m in enumerate(models):
            parts = (m[0], m[1], m[2], m[3])
            for k in range(4):
                a = np.asarray(parts[k])
                if a.size != sizes[k]:
                    raise ValueError("all models must share the first model's shapes")
                np.copyto(self.views[i][k], a.reshape(-1), casting="unsafe")
        if self._sh is None or self._sh[0] is not st:
            self._sh = (st, int(st.cuda_stream))
        sh = self._sh[1]
        lib = self.lib
        from .. import _lib
        _lib.check("cfa_memcpy_async", lib.cfa_memcpy_async(self.dev_ptr, self.host_ptr, 4 * self.total, sh))
        _lib.check(self.name, self.fn(*self.args, sh))
        _lib.check("cfa_stream_synchronize", lib.cfa_stream_synchronize(sh))
        g = self.out.numpy()[:self.M * self.P].reshape(self.M, self.P).copy()
        offs, shapes = self.offs, self.shapes
        return [[g[i, offs[k]:offs[k + 1]].reshape(shapes[k]) for k in range(4)] for i in range(self.M)]


def gradients_batched(ml_model: int, x, y, models: Sequence, stride: int = 1, device=None) -> List[list]:
    """Gradients of the device's cost at every model of ``models`` (list of (W1, b1, W2, b2)),
    in ONE kernel launch. x, y and the models are packed into one pinned staging buffer (one
    H2D); the kernel writes the gradients straight into pinned host memory. Everything but the
    pack, the copy, the launch and the unpack is prepared once per shape (``_GradPlan``).
    Returns one list of four fp32 arrays per model."""
    if not models:
        return []
    from ._runtime import mixer
    hm = mixer() if device is None else None
    eng = hm.engine if hm is not None else get_engine(device)
    W1 = np.asarray(models[0][0])
    shapes = (W1.shape, (int(np.size(models[0][1])),), np.asarray(models[0][2]).shape,
              (int(np.size(models[0][3])),))
    M = len(models)
    x = np.asarray(x)
    y = np.asarray(y)
    if x.ndim != 2 or y.ndim != 2 or x.shape[0] != y.shape[0]:
        raise ValueError("x must be [B, inputs] and y [B, classes]")
    if ml_model == 1:
        if W1.ndim != 3 or W1.shape[1] != 1:
            raise ValueError("CNN W1 must be [filter, 1, number]")
        geom = {"filter": W1.shape[0], "number": W1.shape[2], "stride": int(stride)}
    elif ml_model == 2:
        geom = {"intermediate_nodes": W1.shape[1]}
    else:
        raise ValueError("Unable to set the ML model paramters")
    key = (ml_model, shapes, M, x.shape, y.shape, tuple(sorted(geom.items())))
    if hm is not None:
        st = hm._stream()
        plans = getattr(hm._tls, "grad_plans", None)
        if plans is None:
            plans = hm._tls.grad_plans = {}
    else:
        st = _STREAMS.get(eng.device)
        if st is None:  # one stream per device for calls without a HostMixer, not one per call
            st = _STREAMS[eng.device] = torch.cuda.Stream(eng.device)
        plans = {}
    plan = plans.get(key)
    if plan is None:
        if len(plans) >= 8:
            plans.pop(next(iter(plans)))
        P = sum(int(np.prod(sh)) for sh in shapes)
        if ml_model == 1:
            L2 = -(-(-(-x.shape[1] // stride)) // stride)
            if P != geom["filter"] * geom["number"] + geom["number"] + L2 * geom["number"] * y.shape[1] + y.shape[1]:
                raise ValueError("CNN bucket size does not match the geometry")
        elif P != x.shape[1] * geom["intermediate_nodes"] + geom["intermediate_nodes"] + \
                geom["intermediate_nodes"] * y.shape[1] + y.shape[1]:
            raise ValueError("2NN bucket size does not match the geometry")
        plan = plans[key] = _GradPlan(eng, ml_model, shapes, M, x.shape, y.shape, geom)
    return plan.run(x, y, models, st)


def gradients(ml_model: int, x, y, W1, b1, W2, b2, stride: int = 1, device=None) -> list:
    """``gradients_batched`` for one model."""
    return gradients_batched(ml_model, x, y, [(W1, b1, W2, b2)], stride=stride, device=device)[0]
