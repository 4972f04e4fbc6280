"""Drop-in for FL_radar_dataset/consensus/consensus_v4.py: as the radar consensus_v3, but the
neighbour argument is a single device id (the ring neighbour) read for each of the `neighbors`
iterations (:88-89)."""
from __future__ import annotations

import warnings

from .consensus_v3 import CFA_process as _RadarV3


class CFA_process(_RadarV3):
    def federated_weights_computing(self, neighbor, neighbors, epoch_count, eps_t_control, epoch=0, max_lag=30):
        warnings.filterwarnings("ignore")
        loaded = self._collect_v3([neighbor] * neighbors, neighbors, epoch_count, max_lag,
                                  "results/dump_train_model{}.npy")
        return self._apply_weights(loaded)
