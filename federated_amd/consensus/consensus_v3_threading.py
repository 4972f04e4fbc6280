"""Drop-in for ``consensus.consensus_v3_threading`` (tensorflow2_implementations/CIFAR100_dataset/
consensus/consensus_v3_threading.py): consensus_v3 with a caller-supplied lock held around the
mixing step (:147-161). The libcfa call itself is re-entrant (no global state; ctypes releases
the GIL), so the lock only serialises what the reference serialises."""
from __future__ import annotations

import warnings

from ._tf2 import TF2Base


class CFA_process(TF2Base):
    count_key = "epoch_count"

    def __init__(self, fun_lock, devices, ii_saved_local, neighbors, federated=True, graph=0):
        self.fun_lock = fun_lock
        super().__init__(devices, ii_saved_local, neighbors, federated, graph)

    def federated_weights_computing(self, neighbor, neighbors, epoch_count, eps_t_control, epoch=0, max_lag=30):
        warnings.filterwarnings("ignore")
        loaded = self._collect_v3(neighbor, neighbors, epoch_count, max_lag,
                                  "results/dump_train_model{}.npy")
        with self.fun_lock:
            return self._apply_weights(loaded)
