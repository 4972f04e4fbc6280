"""Drop-in for ``consensus.consensus_v4`` (tensorflow2_implementations/MNIST_dataset/consensus/
consensus_v4.py; identical in CIFAR100 and CIFAR_crossentropy). Adds ``get_neighbor_weights``,
the ring rule for N < 2 (in-neighbour ii-1, out-neighbour ii+1) and a gradient mix that uses the
caller's eps. Reference call site: ..._CIFAR100_gradients_exchange.py:393-457.
"""
from __future__ import annotations

import warnings

import numpy as np

from ._runtime import pause
from ._tf2 import TF2Base, _mix_into, kregular_ring, to_tensors, tx_ring


class CFA_process(TF2Base):
    count_key = "epoch_count"

    def get_neighbor_weights(self, epoch_count, outfile, outfile_models, epoch=0, max_lag=1):
        """consensus_v4.py:30-95, on the shared protocol helpers of ``TF2Base``: status poll
        (one retry), ``pause(round(np.random.random(), 2))`` (drawn even after a failed status
        read, as the reference does), staleness wait, model load with one retry. Returns
        (model, success)."""
        warnings.filterwarnings("ignore")
        ok, nbr_count = self._read_status(outfile)
        pause(round(np.random.random(), 2))
        if not ok:
            return [], False
        return self._wait_and_load(outfile, outfile_models, nbr_count, epoch_count, max_lag)

    def get_connectivity(self, ii_saved_local, neighbors, devices):
        """consensus_v4.py:111-141."""
        return kregular_ring(ii_saved_local, neighbors, devices)

    def get_tx_connectivity(self, ii_saved_local, neighbors, devices):
        """consensus_v4.py:143-173 (uses self.devices for the wrap, as the reference)."""
        return tx_ring(ii_saved_local, neighbors, self.devices)

    def _collect_v4(self, neighbor, neighbors, epoch_count, model_tpl):
        """consensus_v4.py:184-199 / :225-244 (max_lag is fixed to 1 there)."""
        loaded = []
        if neighbors > 1:
            for q in range(neighbors):
                outfile_models = model_tpl.format(neighbor[q])
                outfile = "results/dump_train_variables{}.npz".format(neighbor[q])
                w, ok = self.get_neighbor_weights(epoch_count, outfile, outfile_models, epoch=0, max_lag=1)
                if ok:
                    loaded.append(w)
                if self.training_end and len(loaded) > 0:
                    break
        else:
            outfile_models = model_tpl.format(neighbor)
            outfile = "results/dump_train_variables{}.npz".format(neighbor)
            w, ok = self.get_neighbor_weights(epoch_count, outfile, outfile_models, epoch=0, max_lag=1)
            if ok:
                loaded.append(w)
        return loaded

    def federated_weights_computing(self, neighbor, neighbors, epoch_count, eps_t_control, epoch=0, max_lag=30):
        """consensus_v4.py:176-217 (eps overridden to 1/(n_loaded + 1), :203)."""
        warnings.filterwarnings("ignore")
        loaded = self._collect_v4(neighbor, neighbors, epoch_count, "results/dump_train_model{}.npy")
        return self._apply_weights(loaded)

    def federated_grads_computing(self, neighbor, neighbors, epoch_count, eps_t_control, max_lag=1):
        """consensus_v4.py:219-260: the caller's eps_t_control is used (no override, :248)."""
        warnings.filterwarnings("ignore")
        loaded = self._collect_v4(neighbor, neighbors, epoch_count, "results/dump_train_grad{}.npy")
        if len(loaded) > 0:
            _mix_into(self.local_gradients, loaded, eps_t_control)
        return to_tensors([self.local_gradients[ii] for ii in range(self.layers)])
