"""ORACLE — TEST INFRASTRUCTURE ONLY. Not part of the product.

CPU (numpy) restatement of the reference's consensus arithmetic, used as the parity checker
for the HIP kernels in ``libcfa.so``. Only ``tests/``, ``__graft_entry__.smoke()``,
``bench.py``'s ``cpu_baseline`` leg and the measurement scripts under ``tools/`` (the numpy
column of their tables) may import this module, and only as the checker or as the timed CPU
baseline. The product path (``federated_amd``) never imports it.

Each function restates one reference code path with the same operation order and the same
numpy dtype rules (numpy 2 / NEP 50 promotion), citing the reference file:line it follows
(paths under labRadioVision/federated; TF1 = tensorflow1_implementations,
TF2 = tensorflow2_implementations/MNIST_dataset unless stated).

Pinning: every function here is checked against golden vectors produced by running the
reference code itself (``tests/golden/make_golden.py``) in ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
import random
from typing import List, Sequence

import numpy as np

# ----------------------------------------------------------------------------------------
# Generic sequential rule (the TF2 idiom, fp32 in / fp32 out)
# ----------------------------------------------------------------------------------------


def sequential_mix(local: np.ndarray, nbrs: Sequence[np.ndarray], alphas: Sequence[float]) -> np.ndarray:
    """w <- w + a_j * (x_j - w) for j in order (TF2 consensus_v3.py:153-155).

    ``a_j`` are Python floats, so under NEP 50 they are cast to the array dtype (fp32 for fp32
    buckets) exactly as in the reference."""
    w = local
    for x, a in zip(nbrs, alphas):
        w = w + a * (x - w)
    return w


def closed_form_coeffs(alphas: Sequence[float]) -> List[float]:
    """Coefficients of out = c0*local + sum_j c_{j+1} x_j equal to the sequential rule:
    c0 = prod(1 - a_j), c_{j+1} = a_j * prod_{k>j} (1 - a_k)."""
    n = len(alphas)
    c = [0] * (n + 1)
    tail = 1
    for j in range(n - 1, -1, -1):
        c[j + 1] = alphas[j] * tail
        tail *= 1 - alphas[j]
    c[0] = tail
    return c


# ----------------------------------------------------------------------------------------
# TF2 consensus_v2/v3/v4 (a5, a6)
# ----------------------------------------------------------------------------------------


def tf2_weights(local_layers, nbr_models, training_end: bool = False) -> list:
    """consensus_v3.py:144-159 (= v2 :144-159, v4 :202-217): eps <- 1/(len(nbrs)+1)
    (overrides the argument, :145); if training_end the local model becomes the LAST received
    neighbour (:147-152); else per neighbour q and layer k: w[k] <- w[k] + eps*(x_q[k] - w[k]).
    Returns the list the reference returns (``self.local_weights.tolist()``)."""
    w = list(local_layers)
    if len(nbr_models) > 0:
        eps = 1 / (len(nbr_models) + 1)
        for q in range(len(nbr_models)):
            if training_end:
                for k in range(len(w)):
                    w[k] = nbr_models[-1][k]
                break
            for k in range(len(w)):
                w[k] = w[k] + eps * (nbr_models[q][k] - w[k])
    return w


def tf2_grads_v3(local_grads, nbr_grads) -> list:
    """consensus_v3.py:232-245: eps <- 1/(len+1) (override, :233), sequential rule per layer."""
    g = list(local_grads)
    if len(nbr_grads) > 0:
        eps = 1 / (len(nbr_grads) + 1)
        for q in range(len(nbr_grads)):
            for k in range(len(g)):
                g[k] = g[k] + eps * (nbr_grads[q][k] - g[k])
    return g


def tf2_grads_v4(local_grads, nbr_grads, eps: float) -> list:
    """consensus_v4.py:247-260: the caller's eps is used as given (the override is commented
    out at :248)."""
    g = list(local_grads)
    for q in range(len(nbr_grads)):
        for k in range(len(g)):
            g[k] = g[k] + eps * (nbr_grads[q][k] - g[k])
    return g


# ----------------------------------------------------------------------------------------
# TF1 consensus package (a1, a2, a3, a4)
# ----------------------------------------------------------------------------------------


def tf1_weight_factor(devices: int, ii: int, ii2: int, denom_neighbors: int) -> np.float64:
    """Equation (11) as coded: b = 1/devices; b_j / (b_j + m * b_i) with m = N-1 in cfa.py:66-68
    and cfa_ge_2stage.py:73-75, m = n (this call's neighbour count) in cfa_ongraphs.py:109-111."""
    b_v = 1 / devices
    balancing_vect = np.ones(devices) * b_v
    return balancing_vect[ii2] / (balancing_vect[ii2] + denom_neighbors * balancing_vect[ii])


def tf1_mix(local4, nbr4_list, eps: float, factors) -> list:
    """Sequential TF1 mix of the 4 tensors (W1, b1, W2, b2) (cfa.py:69-76 and the same lines in
    cfa_ongraphs.py:112-119 / cfa_ge_2stage.py:76-83): w <- w + eps*wf_j*(x_j - w).
    Under numpy 2, ``eps*wf`` is an np.float64, so every step after the first subtraction is
    fp64 (as in the reference). Returns [W1, b1, W2, b2] with biases squeezed
    (cfa.py:141-144)."""
    w = [np.asarray(t) for t in local4]
    for x4, wf in zip(nbr4_list, factors):
        w = [w[k] + eps * wf * (np.asarray(x4[k]) - w[k]) for k in range(4)]
    return [np.asarray(w[0]), np.squeeze(np.asarray(w[1])), np.asarray(w[2]), np.squeeze(np.asarray(w[3]))]


def tf1_mix_flat(local: np.ndarray, nbrs, alphas) -> np.ndarray:
    """tf1_mix on one flat fp32 bucket: w <- w + a_j*(x_j - w) with a_j = eps*wf_j an
    np.float64 (cfa.py:69-76): the first subtraction is fp32, everything after it fp64.
    Returns the fp64 (or, with no neighbour, the fp32 input) result as the reference does."""
    w = np.asarray(local)
    for x, a in zip(nbrs, alphas):
        w = w + np.float64(a) * (np.asarray(x) - w)
    return w


COMPRESSION = {  # cfa_ongraphs.py:227-271: (threshold, replacement, differential)
    1: (0.001, 0.0001, False),
    2: (1.e-4, 1.e-4, True),
    3: (1.e-3, 1.e-3, True),
    4: (0.01, 0.001, False),
}


def tf1_compress(W_up_l2: np.ndarray, n_W_l2: np.ndarray, mode: int):
    """Vectorised restatement of the compression double loop cfa_ongraphs.py:225-273.
    Modifies ``W_up_l2`` in place (as the reference does) and returns counter_param."""
    if mode not in COMPRESSION:
        return W_up_l2.shape[0] * W_up_l2.shape[1]
    thr, rep, diff = COMPRESSION[mode]
    if diff:
        d = W_up_l2 - n_W_l2
        mask = np.abs(d) < thr
        W_up_l2[mask] = n_W_l2[mask] + np.sign(d[mask]) * rep
    else:
        mask = np.abs(W_up_l2) < thr
        W_up_l2[mask] = np.sign(W_up_l2[mask]) * rep
    return int(np.count_nonzero(~mask))


def tf1_datagrad_slice(datagrad4, ii: int) -> list:
    """Slot ``ii`` of a neighbour's datagrad tensors (cfa_ge_2stage.py:575-589): the weight
    gradients are [..., devices] arrays read as ``g[..., ii]``; the bias gradients are squeezed
    first (:578-579)."""
    return [np.asarray(datagrad4[0])[..., ii], np.squeeze(np.asarray(datagrad4[1]))[..., ii],
            np.asarray(datagrad4[2])[..., ii], np.squeeze(np.asarray(datagrad4[3]))[..., ii]]


def tf1_mewma(W4, states4, grads4_list, rho: float, lr1: float, lr2: float,
              use_filtered: bool, init: bool) -> list:
    """CFA-GE gradient step (cfa_ge_2stage.py:591-621 fast; :329-371 4-stage), for neighbour
    j in order with its slot-ii gradients ``grads4_list[j]`` = [gW1, gb1, gW2, gb2]:
      s_j <- g_j (4-stage, epoch 1: init=True) or rho*g_j + (1-rho)*s_j (MEWMA);
      W   <- W - lr * (s_j if use_filtered else g_j), lr = lr1 (layer 1) / lr2 (layer 2).
    ``states4`` are the caller's [..., N] saved-state arrays, updated in place at slot j.
    use_filtered: CNN fast path only (:603-606); 2NN fast (:618-621) and 4-stage (:347-350)
    subtract the raw gradient."""
    W = list(W4)
    lrs = (lr1, lr1, lr2, lr2)
    for j, g4 in enumerate(grads4_list):
        for k in range(4):
            g = g4[k]
            s = states4[k]
            if init:
                s[..., j] = g
            else:
                s[..., j] = rho * g + (1 - rho) * s[..., j]
            W[k] = W[k] - lrs[k] * (s[..., j] if use_filtered else g)
    return W


# ----------------------------------------------------------------------------------------
# Neighbour selection (a7)
# ----------------------------------------------------------------------------------------


def tf1_kregular(ii: int, neighbors: int, devices: int) -> np.ndarray:
    """cfa.py:14-32 (identical in cfa_ongraphs.py:54-72, cfa_ge_2stage.py:14-32)."""
    if ii == 0:
        return np.arange(ii + 1, ii + neighbors + 1)
    if ii == devices - 1:
        return np.arange(ii - neighbors, ii)
    if ii >= math.ceil(neighbors / 2) and ii <= devices - math.ceil(neighbors / 2) - 1:
        s = np.arange(ii - math.floor(neighbors / 2), ii + math.floor(neighbors / 2) + 1)
    elif ii - math.ceil(neighbors / 2) < 0:
        s = np.arange(0, neighbors + 1)
    else:
        s = np.arange(devices - neighbors - 1, devices)
    return np.delete(s, np.where(s == ii))


def tf2_kregular_v3(ii: int, neighbors: int, devices: int) -> np.ndarray:
    """consensus_v3.py:44-70: at least 2 neighbours."""
    return tf1_kregular(ii, max(neighbors, 2), devices)


def tf2_kregular_v4(ii: int, neighbors: int, devices: int):
    """consensus_v4.py:111-141: N < 2 -> ring in-neighbour ii-1 (0 -> devices-1), a scalar."""
    if neighbors < 2:
        return ii - 1 if ii > 0 else devices - 1
    return tf1_kregular(ii, neighbors, devices)


def tf2_tx_v4(ii: int, neighbors: int, devices: int):
    """consensus_v4.py:143-173: N < 2 -> ring out-neighbour ii+1 (devices-1 -> 0)."""
    if neighbors < 2:
        return 0 if ii == devices - 1 else ii + 1
    return tf1_kregular(ii, neighbors, devices)


def mobile_neighbors(graph: np.ndarray, ii: int, max_neighbors: int, devices: int, g: int) -> np.ndarray:
    """cfa_ongraphs.py:33-52: row ii of adjacency g, then random.choices(k=max) (WITH
    replacement, Python ``random``) if there are more than max_neighbors."""
    row = graph[ii, :, g]
    nb = np.asarray([kk for kk in range(devices) if row[kk] == 1], dtype=np.uint8)
    if nb.size > max_neighbors:
        return np.asarray(random.choices(nb, k=max_neighbors))
    return nb


# ----------------------------------------------------------------------------------------
# FedAvg parameter server (f1)
# ----------------------------------------------------------------------------------------


def ps_fedavg(params, models, update_factor, divide: bool = True) -> list:
    """parameter_server_v2.py:159-161 / parameter_server.py:154, :74:
    p[q] <- p[q] + u * (x_k[q] - p[q]) / C for k in order (C = number of received models);
    the transfer-learning branch (:150-157) omits the division (divide=False)."""
    p = list(params)
    C = len(models)
    for q in range(len(p)):
        for k in range(C):
            if divide:
                p[q] = p[q] + update_factor * (models[k][q] - p[q]) / C
            else:
                p[q] = p[q] + update_factor * (models[k][q] - p[q])
    return p


# ----------------------------------------------------------------------------------------
# f1: aggregation loops embedded in the reference's drivers
# ----------------------------------------------------------------------------------------
def ps_mqtt_aggregate(model_parameters, local_models_storage, active_device_indexes, update_factor, active):
    """TF2/FL_over_MQTT/PS_server.py:130-133."""
    mp = list(model_parameters)
    for q in range(len(mp)):
        for k in range(active):
            mp[q] = mp[q] + update_factor * (local_models_storage[active_device_indexes[k]][q] - mp[q]) / active
    return mp


def learner_consensus_mix(model_parameters, rx_global_model, update_factor=1, active=2):
    """TF2/FL_over_MQTT/learner_consensus.py:151-152."""
    mp = list(model_parameters)
    for q in range(len(mp)):
        mp[q] = mp[q] + update_factor * (rx_global_model[q] - mp[q]) / active
    return mp


_KEYS4 = ("weights1", "biases1", "weights2", "biases2")


def cfa_fa_server_init(server4, contents, balancing_vect):
    """TF1/federated_sample_CNN_CFA_FA.py:86-89, devices in order."""
    s = list(server4)
    for d, c in enumerate(contents):
        for k, key in enumerate(_KEYS4):
            s[k] = s[k] + balancing_vect[d] * c[key]
    return s


def cfa_fa_server_round(server4, contents, eps_t_control, balancing_vect):
    """TF1/federated_sample_CNN_CFA_FA.py:130-133 (same as :103-110), devices in order."""
    s = list(server4)
    for d, c in enumerate(contents):
        for k, key in enumerate(_KEYS4):
            s[k] = s[k] + eps_t_control * balancing_vect[d] * (c[key] - s[k])
    return s


def cfa_fa_client_mix(W_val_l1, b_val_l1, W_val_l2, b_val_l2, mathcontent, eps_t_control2):
    """TF1/federated_sample_CNN_CFA_FA.py:280-283."""
    W_val_l1 = W_val_l1 + eps_t_control2 * (np.asarray(mathcontent['weights1']) - W_val_l1)
    b_val_l1 = b_val_l1 + eps_t_control2 * (np.squeeze(np.asarray(mathcontent['biases1'])) - b_val_l1)
    W_val_l2 = W_val_l2 + eps_t_control2 * (np.array(mathcontent['weights2']) - W_val_l2)
    b_val_l2 = b_val_l2 + eps_t_control2 * (np.squeeze(np.asarray(mathcontent['biases2'])) - b_val_l2)
    return W_val_l1, b_val_l1, W_val_l2, b_val_l2


# ----------------------------------------------------------------------------------------
# (f2) MQTT payloads: the reference's own codec is CPython's stdlib pickle (3.10.12 here),
# applied to the dicts the drivers build. These restate the driver lines with that codec.
# ----------------------------------------------------------------------------------------


def mqtt_learner_payload(model_list, device_index, frame_count, epoch_count, training_end) -> bytes:
    """TF2/FL_over_MQTT/learner_consensus.py:260-268: layer lists via tolist(), then device,
    framecount, local_epoch, training_end; pickle.dumps with the default protocol."""
    import pickle
    detObj = {}
    for k in range(len(model_list)):
        detObj['model_layer{}'.format(k)] = model_list[k].tolist()
    detObj['device'] = device_index
    detObj['framecount'] = frame_count
    detObj['local_epoch'] = epoch_count
    detObj['training_end'] = training_end
    return pickle.dumps(detObj)


def mqtt_ps_payload(model_list, epoch_count, training_end_signal) -> bytes:
    """TF2/FL_over_MQTT/PS_server.py:140-145 (published at :146-149)."""
    import pickle
    detObj = {}
    for k in range(len(model_list)):
        detObj['global_model_layer{}'.format(k)] = model_list[k].tolist()
    detObj['global_epoch'] = epoch_count
    detObj['training_end'] = training_end_signal
    return pickle.dumps(detObj)


def mqtt_decode_layers(payload: bytes, layers: int, prefix: str = 'model_layer') -> list:
    """learner_consensus.py:136-144 / PS_server.py:90, 116-117: pickle.loads, then
    np.asarray per layer list (fp64 for tolist() floats)."""
    import pickle
    st = pickle.loads(payload)
    return [np.asarray(st['{}{}'.format(prefix, k)]) for k in range(layers)]


def mqtt_learner_receive(model_parameters, payload: bytes, layers: int):
    """learner_consensus.py:136-153: decode; training_end -> the received model, else
    p + 1 * (rx - p) / 2 per layer. Returns (weights, global_epoch, training_end)."""
    import pickle
    st = pickle.loads(payload)
    rx = [np.asarray(st['model_layer{}'.format(k)]) for k in range(layers)]
    if st['training_end']:
        return rx, st['local_epoch'], True
    return learner_consensus_mix(list(model_parameters), rx, 1, 2), st['local_epoch'], False


# ----------------------------------------------------------------------------------------
# (f3) CFA-GE neighbour-gradient evaluation: the TF1 graphs of cfa_ge_2stage.py:391-433 with
# their gradients derived by hand (float64, from the fp32 values the placeholders receive).
# Pinned by central finite differences and by torch autograd in tests/test_tf1_models.py.
# ----------------------------------------------------------------------------------------


def _tf_same_left(L: int, k: int, s: int) -> int:
    out = -(-L // s)
    return max((out - 1) * s + k - L, 0) // 2


def _softmax_xent_grad(logits, y):
    """cost = mean_b(-sum_c y*log(clip(softmax, 1e-15, 0.99))) (:425-426) and d cost/d logits;
    the clip passes the gradient where 1e-15 <= pred <= 0.99 (tf.clip_by_value)."""
    z = logits - logits.max(axis=1, keepdims=True)
    e = np.exp(z)
    pred = e / e.sum(axis=1, keepdims=True)
    B = logits.shape[0]
    clipped = np.clip(pred, 1e-15, 0.99)
    cost = np.mean(-np.sum(y * np.log(clipped), axis=1))
    dpred = np.where((pred >= 1e-15) & (pred <= 0.99), -(y / clipped) / B, 0.0)
    dlogits = (dpred - np.sum(dpred * pred, axis=1, keepdims=True)) * pred
    return cost, dlogits


def tf1_cnn_forward(x, W1, b1, W2, b2, stride):
    """ML_model 1 (:392-405): conv1d SAME (stride S) + bias + relu -> max_pooling1d(S, S, SAME)
    -> NWC flatten -> logits. Returns (logits, pooled [B, L2, NC], argmax positions)."""
    x = np.asarray(x, np.float64)
    W1 = np.asarray(W1, np.float64)
    F, NC = W1.shape[0], W1.shape[2]
    B, L = x.shape
    S = int(stride)
    L1 = -(-L // S)
    L2 = -(-L1 // S)
    pl, ql = _tf_same_left(L, F, S), _tf_same_left(L1, S, S)
    xpad = np.zeros((B, (L1 - 1) * S + F))
    lo = pl
    xpad[:, lo:lo + L] = x[:, :max(0, min(L, xpad.shape[1] - lo))]
    idx = np.arange(L1)[:, None] * S + np.arange(F)[None, :]          # [L1, F]
    z = np.einsum("blf,fc->blc", xpad[:, idx], W1[:, 0, :]) + np.asarray(b1, np.float64).reshape(-1)
    h = np.maximum(z, 0.0)                                             # [B, L1, NC]
    pooled = np.empty((B, L2, NC))
    arg = np.empty((B, L2, NC), dtype=np.int64)
    for q in range(L2):
        ps = [p for p in range(q * S - ql, q * S - ql + S) if 0 <= p < L1]
        win = h[:, ps, :]
        a = np.argmax(win, axis=1)                                     # first maximum
        pooled[:, q, :] = np.take_along_axis(win, a[:, None, :], axis=1)[:, 0, :]
        arg[:, q, :] = np.asarray(ps)[a]
    fc = pooled.reshape(B, L2 * NC)
    logits = fc @ np.asarray(W2, np.float64) + np.asarray(b2, np.float64).reshape(-1)
    return logits, pooled, arg, (xpad, pl, L1)


def tf1_cnn_grads(x, y, W1, b1, W2, b2, stride):
    """d cost / d (W1, b1, W2, b2) of the CNN graph (:392-405, :425-430), float64."""
    W1 = np.asarray(W1, np.float64)
    W2 = np.asarray(W2, np.float64)
    y = np.asarray(y, np.float64)
    F, NC = W1.shape[0], W1.shape[2]
    S = int(stride)
    logits, pooled, arg, (xpad, pl, L1) = tf1_cnn_forward(x, W1, b1, W2, b2, stride)
    B, L2, _ = pooled.shape
    cost, dlog = _softmax_xent_grad(logits, y)
    fc = pooled.reshape(B, -1)
    gW2 = fc.T @ dlog
    gb2 = dlog.sum(axis=0)
    dfc = (dlog @ W2.T).reshape(B, L2, NC) * (pooled > 0)              # relu gradient at the max
    gW1 = np.zeros((F, 1, NC))
    for k in range(F):
        xs = np.take_along_axis(xpad, (arg * S + k).reshape(B, -1), axis=1).reshape(B, L2, NC)
        gW1[k, 0, :] = np.sum(dfc * xs, axis=(0, 1))
    gb1 = dfc.sum(axis=(0, 1))
    return [gW1, gb1, gW2, gb2], cost


def tf1_2nn_grads(x, y, W1, b1, W2, b2):
    """d cost / d (W1, b1, W2, b2) of the 2NN graph (:407-420, :425-430), float64."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    W1 = np.asarray(W1, np.float64)
    W2 = np.asarray(W2, np.float64)
    act = np.maximum(x @ W1 + np.asarray(b1, np.float64).reshape(-1), 0.0)
    logits = act @ W2 + np.asarray(b2, np.float64).reshape(-1)
    cost, dlog = _softmax_xent_grad(logits, y)
    dz = (dlog @ W2.T) * (act > 0)
    return [x.T @ dz, dz.sum(axis=0), act.T @ dlog, dlog.sum(axis=0)], cost


def tf1_flat_shapes(ml_model: int, geom: dict):
    """Per-tensor shapes of a TF1 model bucket (W1, b1, W2, b2) for the CFA-GE graphs."""
    if ml_model == 1:
        L2 = -(-(-(-geom["input_data"] // geom["stride"])) // geom["stride"])
        return [(geom["filter"], 1, geom["number"]), (geom["number"],),
                (L2 * geom["number"], geom["classes"]), (geom["classes"],)]
    return [(geom["input_data"], geom["intermediate_nodes"]), (geom["intermediate_nodes"],),
            (geom["intermediate_nodes"], geom["classes"]), (geom["classes"],)]


def cfa_ge_population_round(W, pub_prev, G_prev, S, lists, x_all, y_all, ml_model, geom, eps, neighbors,
                            rho, lr1, lr2):
    """One 2-stage (fast) CFA-GE round, cfa_ge_2stage.py:388-621, for every device of a
    population, on flat float64 buckets. Device i at epoch e:
      stage 1 (:446-466): mix its local model W[i] with the neighbours' published models
        pub_prev[j] (datamat{j}_{e-1}), alpha = eps * wf(i, j) with m = N-1;
      (:468-471) publish its pre-mix model (the next round's pub[i] = W[i]);
      (:491-535) gradients of its cost (x_all[i], y_all[i]) at each pub_prev[j] -> G_out[i, n];
      (:564-621) for each neighbour n, j in order: slot i of datagrad{j}_{e-1}, i.e.
        G_prev[j, m] with lists[j][m] == i (the last such m, as the slot assignment overwrites;
        zeros if i is not j's neighbour), MEWMA into S[i, n] and the SGD step (filtered for the
        CNN, raw for the 2NN).
    Returns (W_new [D, P], S_new [D, N, P], G_out [D, N, P], pub_new [D, P])."""
    W = np.asarray(W, np.float64)
    D, P = W.shape
    shapes = tf1_flat_shapes(ml_model, geom)
    sizes = [int(np.prod(s)) for s in shapes]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    split = int(offs[2])
    lr = np.where(np.arange(P) < split, lr1, lr2)
    W_new = np.empty_like(W)
    S_new = np.array(S, dtype=np.float64, copy=True)
    G_out = np.zeros((D, max(len(l) for l in lists), P))
    for i in range(D):
        nb = [int(j) for j in lists[i]]
        alphas = [eps * tf1_weight_factor(D, i, j, neighbors - 1) for j in nb]
        w = tf1_mix_flat(np.asarray(W[i], np.float32).astype(np.float64), [np.asarray(pub_prev[j], np.float64) for j in nb],
                         alphas)
        for n, j in enumerate(nb):
            m4 = [np.asarray(pub_prev[j], np.float64)[offs[k]:offs[k + 1]].reshape(shapes[k]) for k in range(4)]
            if ml_model == 1:
                g, _ = tf1_cnn_grads(x_all[i], y_all[i], *m4, stride=geom["stride"])
            else:
                g, _ = tf1_2nn_grads(x_all[i], y_all[i], *m4)
            G_out[i, n] = np.concatenate([a.reshape(-1) for a in g])
        for n, j in enumerate(nb):
            slots = [m for m, k in enumerate(lists[j]) if int(k) == i]
            g = np.asarray(G_prev[j, slots[-1]], np.float64) if slots else np.zeros(P)
            S_new[i, n] = rho * g + (1 - rho) * S_new[i, n]
            w = w - lr * (S_new[i, n] if ml_model == 1 else g)
        W_new[i] = w
    return W_new, S_new, G_out, W.copy()
