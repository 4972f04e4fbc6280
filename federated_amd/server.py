"""Server-side aggregation steps that the reference embeds in its drivers.

The reference's TF2 parameter servers are modules (``consensus/parameter_server*.py``, served by
``federated_amd.consensus``). Three more aggregations live inside driver scripts, which are out of
scope as drivers (argparse, TF graphs, MQTT sockets), but whose arithmetic is this path's fold:

- ``ps_mqtt_aggregate``: FL_over_MQTT ``PS_server.py:130-133``, FedAvg over the decoded payloads;
- ``learner_consensus_mix``: FL_over_MQTT ``learner_consensus.py:151-152``, a device folding the
  received global model;
- ``cfa_fa_server_init``, ``cfa_fa_server_round``, ``cfa_fa_client_mix``: TF1
  ``federated_sample_CNN_CFA_FA.py:86-89``, ``:103-110`` / ``:130-133`` and ``:280-283``.

Each function takes the arrays the reference holds at that point and returns what the cited
lines compute: same dtype, same values, same (broadcast) shapes. In those lines numpy 2
promotes by operand dtype. MQTT payloads decode from ``tolist()`` as fp64, .mat server files are
fp64, and ``balancing_vect[d]`` is an np.float64. So the folds run on fp64 buckets
(``cfa_fold_f64``); a step whose arrays are all fp32 under Python-float scalars runs the fp32
kernels instead, as numpy would keep it in fp32.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from . import _lib
from .consensus._runtime import mixer

__all__ = ["ps_mqtt_aggregate", "learner_consensus_mix", "cfa_fa_server_init", "cfa_fa_server_round",
           "cfa_fa_client_mix"]


def _shapes(local, nbrs):
    out = []
    for k in range(len(local)):
        shp = np.shape(local[k])
        for x in nbrs:
            shp = np.broadcast_shapes(shp, np.shape(x[k]))
        if int(np.prod(shp)) != np.size(local[k]):
            raise ValueError(f"tensor {k}: broadcasting to {shp} changes the element count")
        out.append(shp)
    return out


def _fold(local: Sequence, nbrs: Sequence[Sequence], alphas, rule: int, divisors=None,
          weak_scalars: bool = True) -> List[np.ndarray]:
    """Fold per-layer arrays as numpy 2 would, run of layers by run of layers:
    - every operand fp32 and Python-float scalars: an fp32 chain (fp32 kernels);
    - np.float64 scalars, sequential rule, local and first operand fp32: fp32 first subtraction,
      fp64 after (the TF1 chain, ``cfa_mix_tf1_f64``);
    - otherwise an fp64 chain (``cfa_fold_f64``)."""
    n = len(nbrs)
    shapes = _shapes(local, nbrs)

    def kind(k):
        is32 = lambda a: np.asarray(a).dtype == np.float32
        if n and weak_scalars and rule != _lib.RULE_ACCUMULATE and is32(local[k]) and all(is32(x[k]) for x in nbrs):
            return "f32"
        if n and not weak_scalars and rule == _lib.RULE_SEQUENTIAL and is32(local[k]) and is32(nbrs[0][k]):
            return "tf1"
        return "f64"

    kinds = [kind(k) for k in range(len(local))]
    res: List[np.ndarray] = [None] * len(local)
    k = 0
    while k < len(local):
        e = k
        while e < len(local) and kinds[e] == kinds[k]:
            e += 1
        loc = [np.asarray(local[q]).reshape(-1) for q in range(k, e)]
        nb = [[np.asarray(x[q]).reshape(-1) for q in range(k, e)] for x in nbrs]
        if n == 0:
            outs = [np.array(a, copy=True) for a in loc]
        elif kinds[k] == "f32":
            outs, _ = mixer().mix(loc, nb, alphas, divisors=divisors if rule == _lib.RULE_SEQUENTIAL_DIV else None)
        elif kinds[k] == "tf1":
            outs, _ = mixer().mix_tf1(loc, nb, alphas)
        else:
            outs = mixer().fold64(loc, nb, alphas, rule, divisors)
        for q, o in zip(range(k, e), outs):
            res[q] = np.asarray(o).reshape(shapes[q])
        k = e
    return res


def ps_mqtt_aggregate(model_parameters: Sequence, local_models_storage: Sequence, active_device_indexes,
                      update_factor: float, active: int) -> List[np.ndarray]:
    """PS_server.py:130-133: for every layer q and k < active,
    ``p[q] = p[q] + update_factor * (local_models_storage[idx[k]][q] - p[q]) / active``.
    ``model_parameters`` is ``model_global.get_weights()``; the stored models are the decoded
    payload layers (``np.asarray(list)``, fp64). Returns the new model_parameters list (the
    reference then calls ``set_weights``)."""
    models = [local_models_storage[int(active_device_indexes[k])] for k in range(active)]
    return _fold(list(model_parameters), models, [update_factor] * active, _lib.RULE_SEQUENTIAL_DIV,
                 [active] * active)


def learner_consensus_mix(model_parameters: Sequence, rx_global_model: Sequence, update_factor: float = 1,
                          active: int = 2) -> List[np.ndarray]:
    """learner_consensus.py:151-152: ``p[q] + update_factor * (rx[q] - p[q]) / active`` per layer
    (the reference's values: update_factor 1, active 2)."""
    return _fold(list(model_parameters), [list(rx_global_model)], [update_factor], _lib.RULE_SEQUENTIAL_DIV,
                 [active])


_KEYS = ("weights1", "biases1", "weights2", "biases2")


def _content4(c):
    return [c[k] for k in _KEYS] if isinstance(c, dict) else list(c)


def cfa_fa_server_init(server4: Sequence, contents: Sequence, balancing_vect) -> List[np.ndarray]:
    """federated_sample_CNN_CFA_FA.py:86-89 over every device in order:
    ``server_x = server_x + balancing_vect[devices] * mathcontent[key]`` (``server4`` = the
    np.zeros arrays of :73-76; ``contents[d]`` = device d's loaded datamat content)."""
    bal = np.asarray(balancing_vect)
    return _fold(list(server4), [_content4(c) for c in contents], [bal[d] for d in range(len(contents))],
                 _lib.RULE_ACCUMULATE, weak_scalars=False)


def cfa_fa_server_round(server4: Sequence, contents: Sequence, eps_t_control: float,
                        balancing_vect) -> List[np.ndarray]:
    """federated_sample_CNN_CFA_FA.py:103-110 / :130-133 over every device in order:
    ``server_x = server_x + eps_t_control * balancing_vect[devices] * (mathcontent[key] - server_x)``
    (``eps * b`` is an np.float64)."""
    bal = np.asarray(balancing_vect)
    return _fold(list(server4), [_content4(c) for c in contents],
                 [eps_t_control * bal[d] for d in range(len(contents))], _lib.RULE_SEQUENTIAL,
                 weak_scalars=False)


def cfa_fa_client_mix(W_val_l1, b_val_l1, W_val_l2, b_val_l2, mathcontent, eps_t_control2: float):
    """federated_sample_CNN_CFA_FA.py:280-283: the device pulls its model toward the server's,
    ``W = W + eps2 * (server - W)`` with the server biases squeezed. Returns
    (W_val_l1, b_val_l1, W_val_l2, b_val_l2)."""
    srv = [np.asarray(mathcontent["weights1"]), np.squeeze(np.asarray(mathcontent["biases1"])),
           np.array(mathcontent["weights2"]), np.squeeze(np.asarray(mathcontent["biases2"]))]
    return tuple(_fold([W_val_l1, b_val_l1, W_val_l2, b_val_l2], [srv], [eps_t_control2], _lib.RULE_SEQUENTIAL))
