"""Topology service: the reference's neighbour-selection rules emitted as CSR
tables for the one-launch population kernel (``cfa_mix_population_f32``).

The reference computes each device's neighbour list inside that device's process
(TF1 ``cfa.py:14-32``, ``cfa_ongraphs.py:18-52``; TF2 ``consensus_v3.py:44-70``,
``consensus_v4.py:111-173``) and its mixing coefficients from an eps policy. For a simulated
population resident on one GPU, this module builds, for all D devices at once:

    csr_ptr[D+1], csr_idx[E], csr_coef[E]  (first entry of each row = the device itself)

with the same ordered neighbour lists (the same random draws when the rule is random, using
the same RNG calls) and the same per-step alphas, so one launch reproduces D per-device calls.
"""
from __future__ import annotations

import random
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .consensus import _tf1, _tf2
from ._graphs import RoundGraphs
from .engine import Engine

RULE_SEQUENTIAL = 0
# auto-select the window round above this bucket size: below it the whole population sits in
# the 256 MB Infinity Cache and the single CSR launch already reuses rows (tools/probe/
# window_threshold.py, profiles/r01_window_threshold.jsonl: 32 devices, K = 4: CSR 24.9 vs
# window 34.5 us at P = 262K; window 73 vs CSR 133 us at 1.07M, 123 vs 256 at 2M)
WINDOW_MIN_P = 1 << 19


# -- neighbour lists for every device ---------------------------------------------------------
def kregular_tf1(devices: int, neighbors: int) -> List[List[int]]:
    """cfa.py:14-32 for every device."""
    return [_tf1.kregular(ii, neighbors, devices).tolist() for ii in range(devices)]


def kregular_v3(devices: int, neighbors: int) -> List[List[int]]:
    """consensus_v3.py:44-70 for every device (at least 2 neighbours)."""
    return [_tf2.kregular_v3(ii, neighbors, devices).tolist() for ii in range(devices)]


def ring_v4(devices: int, neighbors: int) -> List[List[int]]:
    """consensus_v4.py:111-141 for every device (N < 2: in-neighbour ii-1)."""
    return [np.atleast_1d(_tf2.kregular_ring(ii, neighbors, devices)).tolist() for ii in range(devices)]


def mobile(graph: np.ndarray, g: int, max_neighbors: Optional[int] = None, devices: Optional[int] = None,
           rng: Optional[random.Random] = None) -> List[List[int]]:
    """Row ii of adjacency ``graph[:, :, g]`` for every device (cfa_mobilenet.py:36-47); with
    ``max_neighbors`` the cfa_ongraphs.py:46-48 draw ``random.choices(k=max_neighbors)`` (with
    replacement) is applied per device in device order, on ``rng`` (default: the global
    ``random`` module, as the reference)."""
    devices = graph.shape[0] if devices is None else devices
    draw = (rng or random).choices
    out = []
    for ii in range(devices):
        row = graph[ii, :, g]
        nb = [kk for kk in range(devices) if row[kk] == 1]
        if max_neighbors is not None and len(nb) > max_neighbors:
            nb = [int(x) for x in draw(np.asarray(nb, dtype=np.uint8), k=max_neighbors)]
        out.append(nb)
    return out


# -- eps policies: per-step alphas of the sequential rule -------------------------------------
def alphas_tf2(nbrs: Sequence[int], ii: int, devices: int) -> List[float]:
    """TF2 weights (consensus_v3.py:145): eps = 1/(n+1) for every step."""
    n = len(nbrs)
    return [1 / (n + 1)] * n


def alphas_tf1_cfa(eps: float, neighbors: int) -> Callable:
    """cfa.py:66-69: eps * b/(b + (N-1) b) with N the configured neighbour count."""
    return lambda nbrs, ii, devices: [eps * _tf1.weight_factor(devices, ii, int(j), neighbors - 1) for j in nbrs]


def alphas_tf1_ongraphs(eps: float) -> Callable:
    """cfa_ongraphs.py:109-113: eps * b/(b + n b) with n this call's neighbour count."""
    return lambda nbrs, ii, devices: [eps * _tf1.weight_factor(devices, ii, int(j), len(nbrs)) for j in nbrs]


def csr(lists: Sequence[Sequence[int]], policy: Callable, devices: Optional[int] = None, coef_dtype=np.float32):
    """(ptr, idx, coef) numpy arrays; row d = [d] + lists[d], coef = [1] + alphas."""
    D = len(lists) if devices is None else devices
    ptr, idx, coef = [0], [], []
    for d, nb in enumerate(lists):
        idx += [d] + [int(j) for j in nb]
        coef += [1.0] + [float(a) for a in policy(nb, d, D)]
        ptr.append(len(idx))
    return (np.asarray(ptr, dtype=np.int32), np.asarray(idx, dtype=np.int32),
            np.asarray(coef, dtype=coef_dtype))


def window_shape(lists: Sequence[Sequence[int]], alphas: Sequence[Sequence[float]], max_side: int = 4):
    """(hl, hr) when every device d's list is the ring window [d-hl .. d-1, d+1 .. d+hr] (mod D)
    in that order and its alphas are one value, else None: such populations mix with
    cfa_mix_window_f32 passes instead of the CSR kernel."""
    D = len(lists)
    if D == 0:
        return None
    nb0 = [int(j) for j in lists[0]]
    for cand_hl in range(0, min(len(nb0), max_side) + 1):
        cand_hr = len(nb0) - cand_hl
        if cand_hr > max_side or cand_hl + cand_hr >= D:
            continue
        ok = True
        for d in range(D):
            want = [(d + o) % D for o in list(range(-cand_hl, 0)) + list(range(1, cand_hr + 1))]
            if [int(j) for j in lists[d]] != want or len(set(float(a) for a in alphas[d])) > 1:
                ok = False
                break
        if ok:
            return cand_hl, cand_hr
    return None


def _zero_on(t: torch.Tensor, stream) -> None:
    """Zero ``t`` in the order of ``stream`` (the stream the kernel that accumulates into it runs
    on; None = the current stream), so the reset cannot race a launch on another stream."""
    if stream is None:
        t.zero_()
        return
    with torch.cuda.stream(stream):
        t.zero_()


class PopulationRound:
    """A population of D device buckets resident in HBM, mixed in ONE launch per round."""

    def __init__(self, engine: Engine, models: torch.Tensor, out: Optional[torch.Tensor] = None):
        if models.dim() != 2 or models.dtype != torch.float32 or not models.is_cuda:
            raise ValueError("models must be a [D, P] fp32 CUDA tensor")
        self.engine = engine
        self.models = models
        self.out = torch.empty_like(models) if out is None else out
        D = models.shape[0]
        dev = models.device
        self.src = torch.tensor([models[d].data_ptr() for d in range(D)], dtype=torch.int64, device=dev)
        self.dst = torch.tensor([self.out[d].data_ptr() for d in range(D)], dtype=torch.int64, device=dev)
        self.tables = None
        self.window = None  # (hl, hr, per-device alphas) when the topology is a ring window
        self._graphs: Optional[RoundGraphs] = None  # captured rounds, rebuilt per topology
        self._parity = 0
        self._tf1 = False

    def set_topology(self, lists, policy, use_window: Optional[bool] = None, numerics: str = "fp32",
                     compression: Optional[Tuple[int, int, int]] = None) -> None:
        """CSR tables for the one-launch population kernel. A ring-window topology with one
        coefficient per device (ring / wrap-around windows under every reference eps policy) can
        run as window passes instead (rows loaded once per 8 devices; same results), all in one
        cfa_mix_ring_round_f32 launch when rows are 16-byte aligned.
        ``use_window=None`` picks the window round only for buckets above WINDOW_MIN_P (512K
        elements); below that the CSR launch reuses rows from the Infinity Cache.
        ``numerics="tf1"``: the TF1 modules' arithmetic (fp32 first subtraction, fp64 chain with
        the fp64 coefficients, one rounding: cfa_mix_population_tf1_f32), for populations run
        with ``alphas_tf1_cfa`` / ``alphas_tf1_ongraphs``; "fp32": the TF2 rule.
        ``compression=(mode, cbegin, cend)`` (TF1 numerics only): the cfa_ongraphs epilogue on
        every device's [cbegin, cend) segment; ``kept`` then holds each device's counter_param
        after a round."""
        if numerics not in ("fp32", "tf1"):
            raise ValueError("numerics must be 'fp32' or 'tf1'")
        self._tf1 = numerics == "tf1"
        if compression is not None and not self._tf1:
            raise ValueError("the compression epilogue belongs to the TF1 (cfa_ongraphs) numerics")
        self._compress = tuple(int(v) for v in compression) if compression else (0, 0, 0)
        self.kept = torch.zeros(self.models.shape[0], dtype=torch.int64, device=self.models.device)
        if use_window is None:
            use_window = self.models.shape[1] > WINDOW_MIN_P
        if self._tf1:
            use_window = False
        D = self.models.shape[0]
        ptr, idx, coef = csr(lists, policy, D, np.float64 if self._tf1 else np.float32)
        dev = self.models.device
        self.tables = tuple(torch.from_numpy(a).to(dev) for a in (ptr, idx, coef))
        alphas = [list(policy(nb, d, D)) for d, nb in enumerate(lists)]
        shape = window_shape(lists, alphas) if use_window else None
        self.window = (shape[0], shape[1], alphas) if shape else None
        # one coefficient per device for the one-launch ring round (the window rule has one)
        self._ring_alphas = (torch.tensor([a[0] if a else 0.0 for a in alphas], dtype=torch.float32, device=dev)
                             if shape else None)
        self._graphs = None

    def run(self, stream=None) -> torch.Tensor:
        """One round: every device's mix of ``models`` into ``out``."""
        self._launch(self.models, self.out, self.src, self.dst, stream)
        return self.out

    def _launch(self, models, out, src, dst, stream=None) -> None:
        if self.tables is None:
            raise RuntimeError("set_topology() first")
        D, P = models.shape
        if self.window is not None:
            hl, hr, alphas = self.window
            if P % 4 == 0:  # 16-byte rows: every pass in one cfa_mix_ring_round_f32 launch
                self.engine.ring_round(out, models, self._ring_alphas, hl, hr, stream)
                return
            for s in range(0, D, 8):
                devs = list(range(s, min(s + 8, D)))
                rows = [models[(s + o) % D] for o in range(-hl, len(devs) + hr)]
                self.engine.mix_window([out[d] for d in devs], rows, [alphas[d] for d in devs], hl, hr, stream)
            return
        if self._tf1:
            mode, cb, ce = self._compress
            if mode:
                _zero_on(self.kept, stream)
            self.engine.population_tf1(dst, src, *self.tables, D, P, stream, mode, cb, ce, self.kept if mode else None)
            return
        self.engine.population(dst, src, *self.tables, D, RULE_SEQUENTIAL, P, stream)

    def rounds(self, R: int, graph: bool = True) -> torch.Tensor:
        """R consecutive rounds on the current stream, each mixing the previous round's output
        (the per-device reference run, repeated: every device's round r reads its neighbours'
        round r-1 models). ``models`` and ``out`` alternate as source and destination; the
        result is left in ``models`` (one extra copy when R is odd) and returned.
        ``graph=True`` replays captured pairs of rounds (hipGraph) instead of launching each
        round from Python; the results are the same bit for bit."""
        if R <= 0:
            return self.models
        if not graph:
            for r in range(R):
                self._step_pair(r & 1)
        else:
            if self._graphs is None:
                self._graphs = RoundGraphs(self.models.device, self._graph_step, 2, lambda: self._parity)
            self._parity = 0
            self._graphs.run(R)
        if R & 1:
            self.models.copy_(self.out)
        return self.models

    def _step_pair(self, parity: int) -> None:
        if parity == 0:
            self._launch(self.models, self.out, self.src, self.dst)
        else:
            self._launch(self.out, self.models, self.dst, self.src)

    def _graph_step(self) -> None:
        self._step_pair(self._parity)
        self._parity ^= 1


class Tf1PopulationRound:
    """A device-resident population on the TF1 protocol (cfa.py:105-154, cfa_ongraphs.py): at
    epoch e every device mixes its own epoch-e model with the models its neighbours PUBLISHED at
    epoch e-1 (their pre-mix inputs of e-1, cfa.py:131-139), with the TF1 numerics (fp64 chain,
    one rounding to fp32: what the driver's fp32 TF variables hold after the assignment).

    Three [D, P] buffers rotate through (current, previous, out): a round mixes current with
    previous into out, then (current, previous, out) <- (out, current, previous). One
    ``cfa_mix_population_tf1_f32`` launch per round over the source table [current | previous]."""

    def __init__(self, engine: Engine, D: int, P: int, device=None, placement_candidates: int = 0):
        """``placement_candidates`` > 3: the three stacks are placement-calibrated
        (``placement.calibrated_rotation``: each stack is in turn read and written, so every
        candidate is scored in both roles) when a stack is 1 GiB or more; ``self.placement``
        holds the probe."""
        dev = engine.device if device is None else torch.device(device)
        self.engine, self.D, self.P = engine, int(D), int(P)
        self.placement = None
        if placement_candidates > 3 and dev.type == "cuda" and self.D * self.P * 4 >= (1 << 30):
            from .placement import calibrated_rotation
            self._bufs, self.placement = calibrated_rotation(3, self.D, self.P, dev, engine, placement_candidates)
            for b in self._bufs:
                b.zero_()
        else:
            self._bufs = [torch.zeros(self.D, self.P, device=dev) for _ in range(3)]
        self._rot = 0
        self._tables = []
        for r in range(3):
            cur, prev, out = (self._bufs[(r + k) % 3] for k in range(3))
            src = torch.tensor([cur[d].data_ptr() for d in range(self.D)] + [prev[d].data_ptr() for d in range(self.D)],
                               dtype=torch.int64, device=dev)
            dst = torch.tensor([out[d].data_ptr() for d in range(self.D)], dtype=torch.int64, device=dev)
            self._tables.append((src, dst))
        self._csr = None
        self._graphs: Optional[RoundGraphs] = None
        self._compress = (0, 0, 0)
        self.kept = torch.zeros(self.D, dtype=torch.int64, device=dev)

    @property
    def current(self) -> torch.Tensor:
        return self._bufs[self._rot]

    @property
    def previous(self) -> torch.Tensor:
        return self._bufs[(self._rot + 1) % 3]

    def set_topology(self, lists, policy, compression: Optional[Tuple[int, int, int]] = None) -> None:
        """Neighbour lists and an eps policy (``alphas_tf1_cfa`` / ``alphas_tf1_ongraphs``); the
        fp64 coefficients go to the device as they are. ``compression=(mode, cbegin, cend)``:
        the cfa_ongraphs epilogue on every device's [cbegin, cend) (its W2 segment); ``kept``
        holds each device's counter_param after a round."""
        self._compress = tuple(int(v) for v in compression) if compression else (0, 0, 0)
        D = self.D
        ptr, idx, coef = [0], [], []
        for d, nb in enumerate(lists):
            idx.append(d)
            coef.append(0.0)
            idx += [D + int(j) for j in nb]
            coef += [float(a) for a in policy(nb, d, D)]
            ptr.append(len(idx))
        dev = self._bufs[0].device
        self._csr = (torch.tensor(ptr, dtype=torch.int32, device=dev), torch.tensor(idx, dtype=torch.int32, device=dev),
                     torch.tensor(coef, dtype=torch.float64, device=dev))

    def load(self, current: torch.Tensor, previous: torch.Tensor) -> None:
        """current [D, P]: every device's epoch-e model; previous [D, P]: the models published at
        epoch e-1."""
        self.current.copy_(current)
        self.previous.copy_(previous)

    def round(self, stream=None) -> None:
        if self._csr is None:
            raise RuntimeError("set_topology() first")
        src, dst = self._tables[self._rot]
        mode, cb, ce = self._compress
        if mode:
            _zero_on(self.kept, stream)
        self.engine.population_tf1(dst, src, *self._csr, self.D, self.P, stream, mode, cb, ce,
                                   self.kept if mode else None)
        self._rot = (self._rot + 2) % 3  # (current, previous, out) <- (out, current, previous)

    def rounds(self, R: int, graph: bool = True) -> None:
        """R rounds; ``graph=True`` replays captured 3-round periods (hipGraph), same results."""
        if not graph:
            for _ in range(R):
                self.round()
            return
        if self._graphs is None:
            self._graphs = RoundGraphs(self._bufs[0].device, self.round, 3, lambda: self._rot)
        self._graphs.run(R)
