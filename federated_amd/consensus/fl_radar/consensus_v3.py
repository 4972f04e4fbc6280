"""Drop-in for FL_radar_dataset/consensus/consensus_v3.py: the MNIST consensus_v3 weight path with
the ring neighbour rule for N < 2 (in-neighbour ii-1, wrap to devices-1; :44-74)."""
from __future__ import annotations

import warnings

from .._tf2 import TF2Base, kregular_ring


class CFA_process(TF2Base):
    count_key = "epoch_count"

    def get_connectivity(self, ii_saved_local, neighbors, devices):
        return kregular_ring(ii_saved_local, neighbors, devices)

    def federated_weights_computing(self, neighbor, neighbors, epoch_count, eps_t_control, epoch=0, max_lag=30):
        warnings.filterwarnings("ignore")
        loaded = self._collect_v3(neighbor, neighbors, epoch_count, max_lag,
                                  "results/dump_train_model{}.npy")
        return self._apply_weights(loaded)
