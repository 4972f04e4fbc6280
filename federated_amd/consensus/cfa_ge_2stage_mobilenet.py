"""Drop-in for ``consensus.cfa_ge_2stage_mobilenet`` (tensorflow1_implementations/consensus/
cfa_ge_2stage_mobilenet.py): CFA-GE on a time-varying network. Differences from cfa_ge_2stage:
neighbours of epoch e are row ii of vGraph.mat graph e (:16-28, :187-192); the saved MEWMA
states are re-created as zeros sized to this round's neighbour count just before the gradient
update (:305-314 and the fast-path twin), so s_j = rho * g_j (fast) / g_j (4-stage epoch 1)."""
from __future__ import annotations

import numpy as np

from . import _tf1
from .cfa_ge_2stage import CFA_ge_process as _CFAGE


class CFA_ge_process(_CFAGE):
    def getMobileNetwork_connectivity(self, ii_saved_local, neighbors, devices, epoch):
        return _tf1.graph_row(ii_saved_local, devices, epoch)

    def __init__(self, federated, devices, ii_saved_local, neighbors, mewma):
        self.federated = federated
        self.devices = devices
        self.ii_saved_local = ii_saved_local
        self.neighbors = neighbors
        self.mewma = mewma
        mat_content = self.getMobileNetwork_connectivity(ii_saved_local, neighbors, devices, 0)
        self.neighbor_vec = np.asarray(mat_content[0], dtype=int)  # :104-105 (first entry only)
        self.grad_fn = None

    def _round_neighbors(self, epoch):
        mat_content = self.getMobileNetwork_connectivity(self.ii_saved_local, self.neighbors, self.devices, epoch)
        print(mat_content)
        self.neighbor_vec = np.asarray(mat_content, dtype=int)
        return self.neighbor_vec

    def _states_for_update(self, states, n):
        shapes = self._grad_shapes()  # [..., devices] -> [..., n]
        return [np.zeros(list(shp[:-1]) + [n]) for shp in shapes]
