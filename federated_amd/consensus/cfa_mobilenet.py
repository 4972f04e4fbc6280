"""Drop-in for ``consensus.cfa_mobilenet`` (tensorflow1_implementations/consensus/cfa_mobilenet.py):
CFA with a time-varying (mobile) network, neighbours of epoch e = row ii of ``vGraph.mat`` graph e.
Mixing math as cfa.py (alpha = eps * b/(b + (N-1) b), N = configured max neighbours)."""
from __future__ import annotations

from . import _tf1
from .cfa import CFA_process as _StaticCFA

import numpy as np


class CFA_process(_StaticCFA):
    def getMobileNetwork_connectivity(self, ii_saved_local, neighbors, devices, epoch):
        """cfa_mobilenet.py:36-47: neighbours of ii in graph[:, :, epoch] (no random draw)."""
        return _tf1.graph_row(ii_saved_local, devices, epoch)

    def __init__(self, federated, devices, ii_saved_local, neighbors):
        # cfa_mobilenet.py:110-116: no neighbour list until the first mixing epoch
        self.federated = federated
        self.devices = devices
        self.ii_saved_local = ii_saved_local
        self.neighbors = neighbors

    def getFederatedWeight(self, n_W_l1, n_W_l2, n_b_l1, n_b_l2, epoch, v_loss, eps_t_control):
        """cfa_mobilenet.py:122-174: as cfa.py, with the neighbour list refreshed from vGraph at
        every mixing epoch (:136-138)."""
        if self.federated and self.devices > 1 and epoch != 0:
            mat_content = self.getMobileNetwork_connectivity(self.ii_saved_local, self.neighbors,
                                                             self.devices, epoch)
            print(mat_content)
            self.neighbor_vec = np.asarray(mat_content, dtype=int)
        return super().getFederatedWeight(n_W_l1, n_W_l2, n_b_l1, n_b_l2, epoch, v_loss, eps_t_control)
