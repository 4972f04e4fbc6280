"""Drop-in for FL_over_MQTT/consensus/consensus_v3.py: consensus_v3's weight path with a
constructor without the `devices` argument (:17). The reference constructor then reads the
undefined name `devices` (:24/:26) and raises NameError; that behaviour is kept, and the
optional keyword `devices` (an extension) makes the class usable."""
from __future__ import annotations

import warnings

from .._tf2 import TF2Base


class CFA_process(TF2Base):
    count_key = "epoch_count"

    def __init__(self, ii_saved_local, neighbors, federated=True, graph=0, *, devices=None):
        if devices is None:
            raise NameError("name 'devices' is not defined")  # consensus_v3.py:24 (MQTT copy)
        super().__init__(devices, ii_saved_local, neighbors, federated, graph)

    def federated_weights_computing(self, neighbor, neighbors, epoch_count, eps_t_control, epoch=0, max_lag=30):
        warnings.filterwarnings("ignore")
        loaded = self._collect_v3(neighbor, neighbors, epoch_count, max_lag,
                                  "results/dump_train_model{}.npy")
        return self._apply_weights(loaded)
