"""Drop-in for ``consensus.cfa`` (tensorflow1_implementations/consensus/cfa.py): CFA on a static
k-regular network. Same class, constructor, methods, argument order and return tuples; the
per-round neighbour mix runs as one libcfa kernel on the GPU.

Reference call site: ``federated_sample_2NN_CFA.py:107,158``
    consensus_p = CFA_process(federated, tot_devices, iii, neighbors_number)
    W1, b1, W2, b2 = consensus_p.getFederatedWeight(n_W_l1, n_W_l2, n_b_l1, n_b_l2, epoch, val_loss, eps)
"""
from __future__ import annotations

import numpy as np

from . import _tf1
from ._runtime import loadmat_retry, pause, savemat_retry, wait_for


class CFA_process:
    def get_connectivity(self, ii_saved_local, neighbors, devices):
        """k-regular neighbour list (cfa.py:14-32)."""
        return _tf1.kregular(ii_saved_local, neighbors, devices)

    def federated_weights_computing2(self, filename, filename2, ii, ii2, epoch, devices, neighbors,
                                     eps_t_control):
        """Single-neighbour step of cfa.py:35-93: mix the working copy in ``filename2`` with the
        neighbour model in ``filename`` (alpha = eps * b/(b + (N-1) b)) and write the result back
        to temp_datamat{ii}_{epoch}.mat. Kept for API compatibility; getFederatedWeight folds all
        neighbours in one GPU pass instead."""
        wait_for(filename2)
        cur = _tf1.model_from_mat(loadmat_retry(filename2))
        wait_for(filename)
        nbr = _tf1.model_from_mat(loadmat_retry(filename))
        a = eps_t_control * _tf1.weight_factor(devices, ii, ii2, neighbors - 1)
        (W1, b1, W2, b2), _ = _tf1.gpu_mix(cur, [nbr], [a])
        savemat_retry("temp_datamat{}_{}.mat".format(ii, epoch),
                      {"weights1": W1, "biases1": b1, "weights2": W2, "biases2": b2})
        return W1, b1, W2, b2

    def __init__(self, federated, devices, ii_saved_local, neighbors):
        self.federated = federated  # true for federation active
        self.devices = devices  # number of devices
        self.ii_saved_local = ii_saved_local  # device index
        self.neighbors = neighbors  # neighbours per device (k-regular degree)
        self.neighbor_vec = self.get_connectivity(ii_saved_local, neighbors, devices)

    def disable_consensus(self, federated):
        self.federated = federated

    def _alphas(self):
        # equation (11) with alpha uses N (configured neighbours), not len(neighbor_vec) (cfa.py:66-68)
        return [_tf1.weight_factor(self.devices, self.ii_saved_local, int(j), self.neighbors - 1)
                for j in self.neighbor_vec]

    def getFederatedWeight(self, n_W_l1, n_W_l2, n_b_l1, n_b_l2, epoch, v_loss, eps_t_control):
        """cfa.py:105-154. Epoch 0 publishes the local model; later epochs mix the local model
        with every neighbour's epoch-1 model (sequential rule, one GPU pass), publish the PRE-mix
        local model as datamat{ii}_{epoch}.mat and return (W1, b1, W2, b2), biases squeezed, as the
        reference's fp64 arrays."""
        ii = self.ii_saved_local
        if not self.federated:
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2, epoch=epoch, loss_sample=v_loss)
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2
        if self.devices <= 1:
            raise _tf1.no_neighbour_error()  # federated with one device: nothing assigns the result (:107, :154)
        if epoch == 0:
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2, epoch=epoch, loss_sample=v_loss)
            return n_W_l1, n_b_l1, n_W_l2, n_b_l2
        models, _, _ = _tf1.load_neighbour_models(self.neighbor_vec, epoch - 1)
        alphas = [eps_t_control * f for f in self._alphas()]
        if not models:  # the reference publishes (:132-139), then reads the unassigned result (:141)
            _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2)
            raise _tf1.no_neighbour_error()
        (W1, b1, W2, b2), _ = _tf1.gpu_mix([n_W_l1, n_b_l1, n_W_l2, n_b_l2], models, alphas)
        _tf1.publish(ii, epoch, n_W_l1, n_b_l1, n_W_l2, n_b_l2)
        return _tf1.squeeze_out(W1, b1, W2, b2)
