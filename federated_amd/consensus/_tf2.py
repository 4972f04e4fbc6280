"""Shared implementation of the TF2 drop-in modules (tensorflow2_implementations/*/consensus).

The TF2 reference publishes each device's Keras weights as ``results/dump_train_model{k}.npy``
(object array of per-layer arrays), its gradients as ``results/dump_train_grad{k}.npy`` and its
status as ``results/dump_train_variables{k}.npz`` (epoch_count / frame_count, training_end);
``federated_weights_computing`` polls those files, then mixes layer by layer with
w[k] <- w[k] + eps * (x_q[k] - w[k]) (consensus_v3.py:73-159).

Here the file protocol is reproduced call for call (including the ``np.random.random()`` draw
inside each ``pause(round(np.random.random(), 2))``, which advances the caller's global numpy RNG
exactly as the reference does), and the mix of all loaded neighbours runs as ONE libcfa kernel
over the flattened model. In fp32 the kernel reproduces numpy's rounding step for step, so the
result is bit-identical to the reference's.
"""
from __future__ import annotations

import os

import numpy as np

from .. import npyfile
from . import _tf1
from ._runtime import mixer, pause


def kregular_v3(ii, neighbors, devices):
    """consensus_v3.py:44-70 (MNIST/CIFAR copies): at least 2 neighbours, k-regular window."""
    return _tf1.kregular(ii, max(neighbors, 2), devices)


def kregular_ring(ii, neighbors, devices):
    """consensus_v4.py:111-141 and FL_radar consensus_v3.py:44-74: N < 2 -> ring in-neighbour
    ii-1 (0 -> devices-1), returned as a scalar; otherwise the k-regular window."""
    if neighbors < 2:
        return ii - 1 if ii > 0 else devices - 1
    return _tf1.kregular(ii, neighbors, devices)


def tx_ring(ii, neighbors, devices):
    """consensus_v4.py:143-173: N < 2 -> ring out-neighbour ii+1 (devices-1 -> 0)."""
    if neighbors < 2:
        return 0 if ii == devices - 1 else ii + 1
    return _tf1.kregular(ii, neighbors, devices)


def _load_vars(outfile, count_key):
    d = npyfile.load(outfile)
    return d[count_key], d["training_end"]


def _mix_into(layers, models, eps):
    """layers[k] <- fold_q(layers[k] + eps * (models[q][k] - layers[k])) for every k, as one GPU
    pass; the results are assigned into ``layers`` (object array) element by element, as the
    reference does (consensus_v3.py:153-155)."""
    local = [np.asarray(layers[k]) for k in range(len(layers))]
    out, _ = mixer().mix(local, [[np.asarray(m[k]) for k in range(len(layers))] for m in models],
                         [eps] * len(models))
    for k in range(len(layers)):
        layers[k] = out[k].reshape(np.shape(local[k]))


class TF2Base:
    """Constructor, topology and state setters common to consensus_v2/v3/v4."""

    count_key = "epoch_count"

    def __init__(self, devices, ii_saved_local, neighbors, federated=True, graph=0):
        self.federated = federated
        self.devices = devices
        self.ii_saved_local = ii_saved_local
        self.neighbors = neighbors
        self.graph = graph
        self.training_end = False
        if graph == 0:
            self.neighbor_vec = self.get_connectivity(ii_saved_local, neighbors, devices)
        else:
            mat_content = self.getMobileNetwork_connectivity(self.ii_saved_local, self.neighbors,
                                                             self.devices, 0)
            self.neighbor_vec = np.asarray(mat_content[0], dtype=int)

    def getMobileNetwork_connectivity(self, ii_saved_local, neighbors, devices, epoch):
        """consensus_v3.py:30-42: row ii of vGraph.mat graph `epoch` (no random draw)."""
        return _tf1.graph_row(ii_saved_local, devices, epoch)

    def get_connectivity(self, ii_saved_local, neighbors, devices):
        return kregular_v3(ii_saved_local, neighbors, devices)

    # -- state setters (consensus_v3.py:247-260) ---------------------------------------------
    def getTrainingStatusFromNeightbor(self):
        return self.training_end

    def update_local_target_model(self, model):
        self.local_weights = model
        self.layers = self.local_weights.size

    def update_local_gradient(self, gradients):
        self.local_gradients = gradients

    def update_local_model(self, model):
        self.local_weights = model
        self.layers = self.local_weights.size

    # -- the file protocol shared by v2/v3 (consensus_v3.py:82-141) and v4 (consensus_v4.py:30-95)
    def _read_status(self, outfile):
        """Poll for a neighbour's status file, load (count, training_end) with one retry.
        Returns (ok, count); ok False after the second failure ("halting federation")."""
        while not os.path.isfile(outfile):
            print("waiting for variables")
            pause(1)
        try:
            nbr_count, self.training_end = _load_vars(outfile, self.count_key)
        except Exception:
            pause(5)
            print("retrying opening variables")
            try:
                nbr_count, self.training_end = _load_vars(outfile, self.count_key)
            except Exception:
                print("halting federation")
                return False, None
        return True, nbr_count

    def _wait_and_load(self, outfile, outfile_models, nbr_count, epoch_count, max_lag, slot=None):
        """Staleness wait (neighbour count < local count - max_lag and not training_end, status
        re-read each second with one retry), then the model load with one retry. Returns
        (model, success). ``slot``: load into a reused buffer (npyfile.load), for models the
        call consumes itself."""
        while not os.path.isfile(outfile_models) or nbr_count < epoch_count - max_lag and not self.training_end:
            pause(1)
            try:
                nbr_count, self.training_end = _load_vars(outfile, self.count_key)
            except Exception:
                pause(2)
                print("retrying opening variables")
                try:
                    nbr_count, self.training_end = _load_vars(outfile, self.count_key)
                except Exception:
                    print("problems loading variables")
        try:
            return npyfile.load(outfile_models, slot=slot), True
        except Exception:
            pause(5)
            print("retrying opening model")
            try:
                return npyfile.load(outfile_models, slot=slot), True
            except Exception:
                print("failed to load model federation")
                return [], False

    def _collect_v3(self, neighbor, neighbors, epoch_count, max_lag, model_tpl):
        """Returns the loaded neighbour models (in order) following the reference loop exactly:
        status file poll, one retry (a second failure stops the loop), ``pause(round(
        np.random.random(), 2))``, staleness wait, model load with one retry, early stop after a
        neighbour that reports training_end."""
        loaded = []
        for q in range(neighbors):
            outfile_models = model_tpl.format(neighbor[q])
            outfile = "results/dump_train_variables{}.npz".format(neighbor[q])
            ok, nbr_count = self._read_status(outfile)
            if not ok:
                break
            pause(round(np.random.random(), 2))
            model, success = self._wait_and_load(outfile, outfile_models, nbr_count, epoch_count, max_lag,
                                                 slot=("tf2", q))
            if success:
                loaded.append(model)
            if self.training_end and len(loaded) > 0:
                break
        return loaded

    def _apply_weights(self, loaded):
        """consensus_v3.py:144-159: eps <- 1/(n+1) (overrides the argument); training_end ->
        copy the last loaded neighbour; else the sequential mix (one GPU pass)."""
        if len(loaded) > 0:
            eps_t_control = 1 / (len(loaded) + 1)
            if self.training_end:
                print("detected training end")
                for k in range(self.layers):  # a copy: the loaded layers live in reused read buffers
                    self.local_weights[k] = np.array(loaded[-1][k])
            else:
                _mix_into(self.local_weights, loaded, eps_t_control)
        return self.local_weights.tolist()


def to_tensors(arrays):
    """``tf.convert_to_tensor`` of each layer when TensorFlow is importable (consensus_v3.py:241-245),
    numpy arrays otherwise."""
    try:
        import tensorflow as tf  # noqa: F401
        return [tf.convert_to_tensor(a) for a in arrays]
    except Exception:
        return [np.asarray(a) for a in arrays]

