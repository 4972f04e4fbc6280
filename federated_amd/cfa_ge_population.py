"""Device-resident CFA-GE population (BASELINE config 3: CNN CFA-GE, 16 devices, one MI355X).

The reference runs each simulated device as its own process and exchanges models and gradients
through .mat files (``federated_sample_CNN_CFA-GE.py:317-319`` starts the processes; the fast
2-stage negotiation is ``cfa_ge_2stage.py:388-621``). Here every device of the population lives
in HBM and one round of the fast negotiation is four steps on the GPU:

1. stage 1 (:446-466): every device mixes its local model with its neighbours' models
   published in the previous round, TF1 coefficients eps * b/(b + (N-1) b);
2. (:468-471) the pre-mix local model becomes the device's published model of this round;
3. (:564-621) every device applies the gradients its neighbours computed for it in the
   previous round (slot i of datagrad{j}_{e-1}): MEWMA filter + SGD step, the neighbours'
   gradient rows passed by pointer (no copy);
4. (:491-535) every device evaluates the gradient of its own cost at each neighbour's
   previous-round model.

Step 4 is ONE ``cfa_ge_grad_{cnn,2nn}_rows_f32`` launch for all D*N (device, neighbour) pairs,
leaving partial sums per batch split; steps 1 and 3 for all devices and the sum of those
partials are ONE ``cfa_ge_population_step_f32`` launch. A round is two launches.

Buckets are fp32 (the population is device-resident; the drop-in modules keep the reference's
fp64 host arithmetic). A round equals ``oracle.cfa_ge_population_round`` within 1e-5 normwise.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._graphs import RoundGraphs
from .consensus import _tf1
from .engine import Engine


def _flat_shapes(ml_model: int, geom: dict, classes: int):
    if ml_model == 1:
        S = int(geom["stride"])
        L2 = -(-(-(-int(geom["input_data"]) // S)) // S)
        return [(geom["filter"], 1, geom["number"]), (geom["number"],), (L2 * geom["number"], classes), (classes,)]
    return [(geom["input_data"], geom["intermediate_nodes"]), (geom["intermediate_nodes"],),
            (geom["intermediate_nodes"], classes), (classes,)]


class CfaGePopulation:
    """D CFA-GE devices resident on one GPU: models, published models, MEWMA states and the
    gradient exchange buffers, advanced one fast-negotiation round per ``round()``."""

    def __init__(self, engine: Engine, ml_model: int, geom: dict, x: torch.Tensor, y: torch.Tensor,
                 lists: Sequence[Sequence[int]], eps: float, neighbors: int, rho: float, lr1: float,
                 lr2: float):
        """``x`` [D, B, L] / ``y`` [D, B, C]: every device's samples and one-hot labels (x_train2,
        y_train2); ``lists``: ordered neighbour lists (``topology.kregular_tf1`` for the reference's
        get_connectivity, cfa_ge_2stage.py:14-32); ``neighbors`` = N of the weight factor."""
        self.engine, self.ml_model, self.geom = engine, int(ml_model), dict(geom)
        dev = engine.device
        D = int(x.shape[0])
        if len(lists) != D or y.shape[0] != D:
            raise ValueError("one neighbour list and one data set per device")
        C = int(y.shape[2])
        self.shapes = _flat_shapes(ml_model, {**geom, "input_data": int(x.shape[2])}, C)
        sizes = [int(np.prod(s)) for s in self.shapes]
        self.P = P = sum(sizes)
        self.lr_split = sizes[0] + sizes[1]
        if P % 4:
            raise ValueError("population rows must be 16-byte aligned (P a multiple of 4)")
        self.D, self.lists = D, [[int(j) for j in l] for l in lists]
        self.N = Nmax = max(1, max(len(l) for l in self.lists))
        self.x, self.y = x, y
        self.rho, self.lr1, self.lr2 = float(rho), float(lr1), float(lr2)
        # state: local models, previous-round published models, MEWMA states, gradients
        self.W = torch.zeros(D, P, device=dev)
        self.pub = torch.zeros(D, P, device=dev)
        self.mixed = torch.empty(D, P, device=dev)
        self.S = torch.zeros(D, Nmax, P, device=dev)
        self.G = torch.zeros(D * Nmax, P, device=dev)       # G[i*N + n]: grad of i's cost at pub[lists[i][n]]
        self.G_next = torch.empty_like(self.G)
        # stage-1 CSR: source table = [W rows | pub rows], local first (cfa.py:66-76 coefficients)
        ptr, idx, coef = [0], [], []
        for i, nb in enumerate(self.lists):
            idx.append(i)
            coef.append(0.0)
            for j in nb:
                idx.append(D + j)
                coef.append(float(np.float32(eps * _tf1.weight_factor(D, i, j, neighbors - 1))))
            ptr.append(len(idx))
        self._csr = (torch.tensor(ptr, dtype=torch.int32, device=dev), torch.tensor(idx, dtype=torch.int32, device=dev),
                     torch.tensor(coef, dtype=torch.float32, device=dev))
        # gradient evaluations: pair (i, n) -> model row lists[i][n] of pub, data row i
        mrow = [j for i, nb in enumerate(self.lists) for j in nb + [0] * (Nmax - len(nb))]
        drow = [i for i, nb in enumerate(self.lists) for _ in range(Nmax)]
        # the gradient launch leaves [M][splits][P] partial sums (each evaluation's batch split over
        # workgroups); the next population-step launch sums them into G_next
        self._splits = engine.grad_splits(len(mrow), int(x.shape[1]), P)
        self._ws = torch.empty(len(mrow) * self._splits * P, device=dev)
        self._mrow = torch.tensor(mrow, dtype=torch.int32, device=dev)
        self._drow = torch.tensor(drow, dtype=torch.int32, device=dev)
        # where device i finds slot i of neighbour j's gradients: G row j*N + m (last m with
        # lists[j][m] == i, as the reference's slot assignment overwrites), or zeros
        self._slot = []
        for i, nb in enumerate(self.lists):
            rows = []
            for j in nb:
                ms = [m for m, k in enumerate(self.lists[j]) if k == i]
                rows.append(j * Nmax + ms[-1] if ms else -1)
            self._slot.append(rows)
        self._refresh_ptrs()

    def _refresh_ptrs(self) -> None:
        """Device pointer tables, uploaded once: (src, dst) for the three rotations of (W, pub,
        mixed) that successive rounds cycle through, and the per-CSR-entry MEWMA state and
        gradient slots for the two parities of the (G, G_next) swap."""
        D, dev = self.D, self.engine.device
        bufs = [self.W, self.pub, self.mixed]
        self._tables = []
        for r in range(3):
            W, pub, mixed = bufs[r % 3], bufs[(r + 1) % 3], bufs[(r + 2) % 3]
            src = torch.tensor([W[d].data_ptr() for d in range(D)] + [pub[d].data_ptr() for d in range(D)],
                               dtype=torch.int64, device=dev)
            dst = torch.tensor([mixed[d].data_ptr() for d in range(D)], dtype=torch.int64, device=dev)
            self._tables.append((src, dst))
        self._bufs, self._rot = bufs, 0
        self._graphs: Optional[RoundGraphs] = None  # captured periods hold these tables
        states, grads = [], ([], [])
        for i, nb in enumerate(self.lists):
            states.append(0)
            grads[0].append(0)
            grads[1].append(0)
            for n in range(len(nb)):
                states.append(self.S[i, n].data_ptr())
                r = self._slot[i][n]
                grads[0].append(self.G[r].data_ptr() if r >= 0 else 0)
                grads[1].append(self.G_next[r].data_ptr() if r >= 0 else 0)
        self._states = torch.tensor(states, dtype=torch.int64, device=dev)
        self._grads = [torch.tensor(g, dtype=torch.int64, device=dev) for g in grads]
        self._gpar = 0

    def load(self, W: torch.Tensor, pub: torch.Tensor, S: Optional[torch.Tensor] = None,
             G: Optional[torch.Tensor] = None) -> None:
        """Set the state: W [D, P] local models, pub [D, P] previous-round published models,
        S [D, N, P] MEWMA states, G [D, N, P] previous-round gradients (G[j, m] = gradient of
        device j's cost at device lists[j][m]'s model)."""
        self.W.copy_(W)
        self.pub.copy_(pub)
        if S is not None:
            self.S.copy_(S)
        if G is not None:
            self.G.copy_(G.reshape(self.G.shape))

    def round(self, stream=None) -> None:
        """One fast-negotiation round for every device (see the module docstring). Afterwards
        W holds the updated models, pub the models published this round, S the MEWMA states and
        G the gradients computed this round."""
        eng, D, P = self.engine, self.D, self.P
        ptr, idx, coef = self._csr
        src, dst = self._tables[self._rot]
        # 4: gradients of every device's cost at its neighbours' previous-round models (partial
        # sums per batch split)
        eng.grad_rows(self.ml_model, self.x, self.y, self.pub, self._mrow, self._drow, None,
                      self.geom, stream, workspace=self._ws)
        # 1 + 3: stage-1 mix and the gradient step with the previous round's gradients, and the
        # sum of this round's partial gradients into G_next, one launch
        eng.ge_population_step(dst, src, self._states, self._grads[self._gpar], ptr, idx, coef, D, self.rho,
                               self.lr1, self.lr2, self.lr_split, self.ml_model == 1, P, stream,
                               reduce=(self._ws, self.G_next, self._splits))
        # 2: the pre-mix local models are this round's published models; the new locals are the
        # updated mixes; this round's gradients become the next round's input
        self._rot = (self._rot + 2) % 3  # (W, pub, mixed) <- (mixed, W, pub)
        b = self._bufs
        self.W, self.pub, self.mixed = b[self._rot], b[(self._rot + 1) % 3], b[(self._rot + 2) % 3]
        self.G, self.G_next = self.G_next, self.G
        self._gpar ^= 1

    def rounds(self, R: int, graph: bool = True) -> None:
        """R consecutive ``round()`` calls on the current stream. ``graph=True`` replays
        captured 6-round periods (the (W, pub, mixed) rotation times the (G, G_next) swap
        returns to its start after 6 rounds) as hipGraphs, so a round costs its kernels and not
        its Python launch path; the results equal R eager rounds bit for bit."""
        if not graph:
            for _ in range(R):
                self.round()
            return
        if self._graphs is None:
            self._graphs = RoundGraphs(self.engine.device, self.round, 6, lambda: (self._rot, self._gpar))
        self._graphs.run(R)

    @property
    def bytes_per_round(self) -> int:
        """HBM bytes of the reduction steps (the stage-1 mixes and the MEWMA updates):
        sum_i (n_i + 2) P * 4 + sum_i (3 n_i + 2) P * 4."""
        return sum((len(nb) + 2) + (3 * len(nb) + 2 if nb else 0) for nb in self.lists) * self.P * 4
