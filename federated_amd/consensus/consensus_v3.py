"""Drop-in for ``consensus.consensus_v3`` (tensorflow2_implementations/MNIST_dataset/consensus/
consensus_v3.py; the CIFAR_crossentropy copy is identical, the CIFAR100 copy is this minus the
gradient method). Reference call site: federated_learning_keras_consensus_FL_threads_CIFAR100.py:307,433,450.
"""
from __future__ import annotations

import warnings

from ._tf2 import TF2Base, _mix_into, to_tensors


class CFA_process(TF2Base):
    count_key = "epoch_count"

    def federated_weights_computing(self, neighbor, neighbors, epoch_count, eps_t_control, epoch=0, max_lag=30):
        """consensus_v3.py:73-159: load up to `neighbors` neighbour models (staleness <= max_lag),
        then mix with eps = 1/(n_loaded + 1) (the argument is overridden, :145); training_end
        copies the last loaded model. Mutates and returns ``self.local_weights`` (as a list)."""
        warnings.filterwarnings("ignore")
        loaded = self._collect_v3(neighbor, neighbors, epoch_count, max_lag,
                                  "results/dump_train_model{}.npy")
        return self._apply_weights(loaded)

    def federated_grads_computing(self, neighbor, neighbors, epoch_count, eps_t_control, epoch=0, max_lag=30):
        """consensus_v3.py:161-245: same loading loop on dump_train_grad{k}.npy; sequential mix
        of the local gradients with eps = 1/(n_loaded + 1) (:233); returns tensors."""
        warnings.filterwarnings("ignore")
        loaded = self._collect_v3(neighbor, neighbors, epoch_count, max_lag,
                                  "results/dump_train_grad{}.npy")
        if len(loaded) > 0:
            _mix_into(self.local_gradients, loaded, 1 / (len(loaded) + 1))
        return to_tensors([self.local_gradients[ii] for ii in range(self.layers)])
