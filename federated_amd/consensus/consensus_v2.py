"""Drop-in for ``consensus.consensus_v2`` (tensorflow2_implementations/*/consensus/consensus_v2.py,
identical in all five dataset directories): consensus_v3's weight path keyed on the neighbours'
``frame_count`` instead of ``epoch_count`` (consensus_v2.py:73-159)."""
from __future__ import annotations

import warnings

from ._tf2 import TF2Base


class CFA_process(TF2Base):
    count_key = "frame_count"

    def federated_weights_computing(self, neighbor, neighbors, frame_count, eps_t_control, epoch=0, max_lag=30):
        warnings.filterwarnings("ignore")
        loaded = self._collect_v3(neighbor, neighbors, frame_count, max_lag,
                                  "results/dump_train_model{}.npy")
        return self._apply_weights(loaded)
