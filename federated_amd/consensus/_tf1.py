"""Pieces shared by the TF1 drop-in modules (cfa, cfa_mobilenet, cfa_ongraphs, cfa_ge_*).

The TF1 reference (tensorflow1_implementations/consensus) exchanges the four tensors
(weights1, biases1, weights2, biases2) of each device through ``datamat{dev}_{epoch}.mat`` files
and mixes them one neighbour at a time, re-reading its working copy from
``temp_datamat{ii}_{epoch}.mat`` between neighbours (cfa.py:35-93, :119-130). Here the neighbour
files are read as the reference reads them (same names, same polling), and all n neighbours are
folded in one GPU pass; the private temp file is not needed.
"""
from __future__ import annotations

import math
import random
from typing import List, Sequence

import numpy as np
import scipy.io as sio

from ._runtime import loadmat_retry, mixer, pause, savemat_retry, wait_for

KEYS = ("weights1", "biases1", "weights2", "biases2")


def kregular(ii: int, neighbors: int, devices: int) -> np.ndarray:
    """k-regular "clamped window" neighbour list (cfa.py:14-32; identical in cfa_ongraphs.py:54-72,
    cfa_ge_2stage.py:14-32): ceil/floor(N/2) on each side of ii, shifted to stay inside
    [0, devices); ii itself removed. Edge devices get N neighbours on one side."""
    if ii == 0:
        return np.arange(ii + 1, ii + neighbors + 1)
    if ii == devices - 1:
        return np.arange(ii - neighbors, ii)
    if math.ceil(neighbors / 2) <= ii <= devices - math.ceil(neighbors / 2) - 1:
        window = np.arange(ii - math.floor(neighbors / 2), ii + math.floor(neighbors / 2) + 1)
    elif ii - math.ceil(neighbors / 2) < 0:
        window = np.arange(0, neighbors + 1)
    else:
        window = np.arange(devices - neighbors - 1, devices)
    return np.delete(window, np.where(window == ii))


def weight_factor(devices: int, ii: int, ii2: int, m: int) -> float:
    """Equation (11) as the reference codes it: b_j / (b_j + m * b_i) with b = 1/devices
    (cfa.py:66-68 with m = N-1; cfa_ongraphs.py:109-111 with m = this call's n). Evaluated in
    float64 with the same operations, so the value (and its fp32 rounding) matches."""
    b = np.ones(devices) * (1 / devices)
    return float(b[ii2] / (b[ii2] + m * b[ii]))


def graph_row(ii: int, devices: int, g: int, path: str = "consensus/vGraph.mat") -> np.ndarray:
    """Neighbours of ii in adjacency tensor ``graph[:, :, g]`` of vGraph.mat (uint8 [dev, dev,
    graphs]); cfa_ongraphs.py:33-44 / cfa_mobilenet.py:36-47 (path relative to cwd, as there)."""
    graph = sio.loadmat(path)["graph"]
    row = graph[ii, :, g]
    return np.asarray([kk for kk in range(devices) if row[kk] == 1], dtype=np.uint8)


def mobile_neighbors(ii: int, max_neighbors: int, devices: int, g: int,
                     path: str = "consensus/vGraph.mat") -> np.ndarray:
    """cfa_ongraphs.py:33-52: the graph row, then ``random.choices(k=max_neighbors)`` (with
    replacement, Python's ``random``) when the row has more than max_neighbors entries."""
    nb = graph_row(ii, devices, g, path)
    if nb.size > max_neighbors:
        return np.asarray(random.choices(nb, k=max_neighbors))
    return nb


def random_neighbors(ii: int, neighbors: int, devices: int) -> np.ndarray:
    """cfa_ongraphs.py:18-31: first `neighbors` entries of np.random.permutation(devices),
    redrawn until ii is not among them."""
    perm = np.random.permutation(devices)
    nb = perm[0:neighbors]
    while np.where(nb == ii)[0].size:
        perm = np.random.permutation(devices)
        nb = perm[0:neighbors]
    return nb


def model_from_mat(content: dict) -> List[np.ndarray]:
    return [np.asarray(content[k]) for k in KEYS]


def load_neighbour_models(nbr_vec, epoch: int, sleep_before: float = 0.0, sleep_after: float = 5.0,
                          temp_path: str = None):
    """Wait for and load datamat{j}_{epoch}.mat for every neighbour j, in order, with the
    reference's protocol sleeps around each (cfa.py:119-130: poll, load, pause(5);
    cfa_ongraphs.py:79 adds pause(2) before the load). Returns (models, extras, wait_time)."""
    models, extras, waited = [], [], 0.0
    for j in np.asarray(nbr_vec).reshape(-1):
        fname = "datamat{}_{}.mat".format(int(j), epoch)
        waited += wait_for(fname) if temp_path is None else wait_for(fname, temp_path)
        if sleep_before:
            pause(sleep_before)
        content = loadmat_retry(fname)
        models.append(model_from_mat(content))
        extras.append(content)
        if sleep_after:
            pause(sleep_after)
    return models, extras, waited


def gpu_mix(local4: Sequence, nbr_models: Sequence, alphas: Sequence[float], compress=None):
    """One GPU pass over all neighbours with the reference's TF1 numerics on fp64 buckets
    (cfa_mix_tf1_f64); returns ([W1, b1, W2, b2] as the reference's fp64 arrays, kept count)."""
    return mixer().mix_tf1(list(local4), nbr_models, alphas, compress)


def no_neighbour_error() -> UnboundLocalError:
    """The error the TF1 modules raise when a mixing epoch has no neighbour, or when a federated
    process is told it is the only device: their result variables are assigned only inside the
    neighbour loop (cfa.py:107-154, the loop :119-130 and its use :141; cfa_ge_2stage.py:189-211
    and :449-463), so Python raises UnboundLocalError. The drop-ins raise the same error at the
    same point of the protocol, so a driver configured that way (N = 1 on the k-regular window
    leaves every interior device without a neighbour, cfa.py:14-32) fails as it does on the
    reference instead of running on with an unmixed model."""
    return UnboundLocalError("local variable 'W_up_l1' referenced before assignment")


def publish(dev: int, ep: int, W1, b1, W2, b2, **extra) -> None:
    """Write datamat{dev}_{ep}.mat with the four tensors plus any extra keys (epoch,
    loss_sample, counter_param), as the reference's savemat calls do."""
    data = {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2}
    data.update(extra)
    savemat_retry("datamat{}_{}.mat".format(dev, ep), data)


def squeeze_out(W1, b1, W2, b2):
    """Return form of the TF1 modules: weights as arrays, biases squeezed (cfa.py:141-144)."""
    return np.asarray(W1), np.squeeze(np.asarray(b1)), np.asarray(W2), np.squeeze(np.asarray(b2))
