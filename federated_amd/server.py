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

from . import _lib, payload as _payload
from .consensus._runtime import mixer

__all__ = ["ps_mqtt_aggregate", "learner_consensus_mix", "cfa_fa_server_init", "cfa_fa_server_round",
           "cfa_fa_client_mix", "ps_mqtt_aggregate_payloads", "ps_mqtt_publish", "learner_consensus_receive",
           "learner_publish"]


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


def _payload_fills(local: Sequence, payloads: Sequence, prefix: str):
    """Per payload, a filler that decodes its layers straight into a pinned fp64 staging row,
    or None when a layer's shape differs from the local one (numpy would broadcast: decode to
    arrays and take the general fold instead)."""
    keys = _payload.layer_keys(prefix, len(local))
    parsed = [p if isinstance(p, _payload.Payload) else _payload.Payload(p) for p in payloads]
    for p in parsed:
        for k, key in enumerate(keys):
            kind, shape = p.info(key)
            if kind == _lib.PAYLOAD_BOOL_ARRAY:
                raise TypeError(f"{key}: boolean layer")  # numpy refuses bool - float subtraction
            if shape != np.shape(local[k]):
                return parsed, None
    return parsed, [lambda dst, p=p: p.read_into(keys, dst) for p in parsed]


def ps_mqtt_aggregate_payloads(model_parameters: Sequence, payloads: Sequence, update_factor: float,
                               active: int, prefix: str = "model_layer") -> List[np.ndarray]:
    """PS_server.py:90-118 + :130-133 from the raw MQTT payloads of the active devices, in
    ``active_device_indexes`` order: each payload's ``model_layer{k}`` lists (what
    ``np.asarray(st['model_layer{k}'])`` gives, fp64) are decoded by the native codec straight
    into the pinned fp64 staging of the fold, then folded on the GPU as ``ps_mqtt_aggregate``
    does. Returns the new model_parameters list (fp64, as the reference's before set_weights)."""
    if len(payloads) != active:
        raise ValueError("one payload per active device")
    local = list(model_parameters)
    parsed, fills = _payload_fills(local, payloads, prefix)
    if fills is None:
        keys = _payload.layer_keys(prefix, len(local))
        return ps_mqtt_aggregate(local, [[p.array(k) for k in keys] for p in parsed], range(active),
                                 update_factor, active)
    return mixer().fold64(local, fills, [update_factor] * active, _lib.RULE_SEQUENTIAL_DIV, [active] * active)


def ps_mqtt_publish(model_list: Sequence, epoch_count: int, training_end_signal: bool) -> bytes:
    """PS_server.py:140-145: ``pickle.dumps({'global_model_layer{k}': w.tolist(), ...,
    'global_epoch': epoch_count, 'training_end': training_end_signal})``, byte for byte."""
    d = {f"global_model_layer{k}": np.asarray(w) for k, w in enumerate(model_list)}
    d["global_epoch"] = int(epoch_count)
    d["training_end"] = bool(training_end_signal)
    return _payload.dumps(d)


def learner_consensus_receive(model_parameters: Sequence, message_payload, update_factor: float = 1,
                              active: int = 2, prefix: str = "model_layer"):
    """learner_consensus.py:136-153 for one received payload: decode ``model_layer{k}`` and
    ``local_epoch``; if ``training_end`` the received model replaces the local one (:146-147),
    else ``p + update_factor * (rx - p) / active`` per layer on the GPU (:149-152). Returns
    (new weights for set_weights, global_epoch, training_end)."""
    p = message_payload if isinstance(message_payload, _payload.Payload) else _payload.Payload(message_payload)
    keys = _payload.layer_keys(prefix, len(model_parameters))
    global_epoch = p.scalar("local_epoch")
    if p.scalar("training_end"):
        return [p.array(k) for k in keys], global_epoch, True
    local = list(model_parameters)
    _, fills = _payload_fills(local, [p], prefix)
    if fills is None:
        return learner_consensus_mix(local, [p.array(k) for k in keys], update_factor, active), global_epoch, False
    return (mixer().fold64(local, fills, [update_factor], _lib.RULE_SEQUENTIAL_DIV, [active]), global_epoch,
            False)


def learner_publish(model_list: Sequence, device_index: int, frame_count: int, epoch_count: int,
                    training_end: bool) -> bytes:
    """learner_consensus.py:261-268: the device's model payload, byte for byte."""
    return _payload.model_payload(model_list, device=device_index, framecount=frame_count,
                                  local_epoch=epoch_count, training_end=training_end)


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
