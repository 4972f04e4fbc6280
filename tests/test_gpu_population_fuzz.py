"""Randomised parity of the one-launch population rounds (topology.PopulationRound) against the
per-device rule, on the GPU.

Each case draws a population and a topology and checks every device's mixed model bit for bit
against the numpy restatement applied device by device (the reference runs one mixing call per
device: TF2 consensus_v3.py:144-157, TF1 cfa.py:69-76 / cfa_ongraphs.py:112-119 and 225-273):

- D from 2 to 40 devices, P from 1 to ~1.5M (rows that are and are not 16-byte multiples, below
  and above the window round's 512K threshold);
- topologies: a ring window (h_left, h_right from 0 to 4: the window and one-launch ring-round
  kernels), random neighbour lists (repeats and the device itself allowed: the CSR kernel),
  k-regular TF1 windows, and devices without neighbours;
- the TF2 eps policy, random per-step alphas, or the TF1 numerics with a cfa_ongraphs
  compression range (every device's counter_param checked);
- one round from ``run`` and two chained rounds from ``rounds(2)`` (graph replay or eager).

CFA_POP_FUZZ_CASES (default 24) sets the number of cases.
"""
import os

import numpy as np
import pytest
import torch

from oracle import cfa_oracle as O

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("CFA_POP_FUZZ_CASES", "24"))
SEED0 = int(os.environ.get("CFA_POP_FUZZ_SEED", "61000"))


def _lists(rng, D):
    r = rng.random()
    if r < 0.4:
        hl, hr = int(rng.integers(0, 5)), int(rng.integers(0, 5))
        while hl + hr >= D:
            hl, hr = max(0, hl - 1), max(0, hr - 1)
        return [[(d + o) % D for o in list(range(-hl, 0)) + list(range(1, hr + 1))] for d in range(D)], "window"
    if r < 0.8:
        return [[int(j) for j in rng.integers(0, D, int(rng.integers(0, 7)))] for _ in range(D)], "random"
    from federated_amd.topology import kregular_tf1
    N = int(rng.integers(1, min(5, D)))
    return kregular_tf1(D, N), "kregular"


def _round_ref(models, lists, alphas, tf1, compression):
    """Every device's mixed model from ``models`` (rows), device by device."""
    out, kept = [], []
    for d, nb in enumerate(lists):
        if tf1:
            y = O.tf1_mix_flat(models[d], [models[j] for j in nb], alphas[d])
            y = y.astype(np.float64) if len(nb) else y.astype(np.float32).copy()
            mode, cb, ce = compression
            if mode:
                seg = y[cb:ce].reshape(1, -1)
                kept.append(O.tf1_compress(seg, models[d][cb:ce].reshape(1, -1), mode))
                y[cb:ce] = seg.reshape(-1)
            out.append(y.astype(np.float32))
        else:
            out.append(O.sequential_mix(models[d], [models[j] for j in nb], alphas[d]).astype(np.float32))
    return np.stack(out), kept


@pytest.mark.parametrize("case", range(CASES))
def test_population_round_fuzz(gpu, case):
    from federated_amd.topology import PopulationRound, alphas_tf2
    rng = np.random.default_rng(SEED0 + case)
    D = int(rng.integers(2, 41))
    r = rng.random()
    P = int(rng.integers(1, 5000)) if r < 0.3 else (int(rng.integers(5000, 400_000)) if r < 0.7
                                                    else int(rng.integers(520_000, 1_500_000)))
    lists, shape = _lists(rng, D)
    tf1 = rng.random() < 0.3
    pol = rng.random()
    if pol < 0.5:
        policy = alphas_tf2
    else:
        table = {d: [float(a) for a in rng.uniform(0.01, 1.0, len(nb))] for d, nb in enumerate(lists)}
        if shape == "window" and rng.random() < 0.7:  # one coefficient per device: the window kernels
            table = {d: [table[d][0]] * len(nb) if nb else [] for d, nb in enumerate(lists)}
        policy = (lambda t: (lambda nb, d, Dn: t[d]))(table)
    alphas = [list(policy(nb, d, D)) for d, nb in enumerate(lists)]
    compression = None
    if tf1 and rng.random() < 0.6:
        cb = int(rng.integers(0, P + 1))
        compression = (int(rng.integers(1, 5)), cb, int(rng.integers(cb, P + 1)))
    models = (rng.standard_normal((D, P)) * 10.0 ** rng.uniform(-3, 0)).astype(np.float32)
    use_window = [None, True, False][int(rng.integers(0, 3))]
    info = (D, P, shape, tf1, compression, use_window)

    dm = torch.from_numpy(models).cuda()
    pr = PopulationRound(gpu, dm)
    pr.set_topology(lists, policy, use_window=use_window, numerics="tf1" if tf1 else "fp32",
                    compression=compression)
    ref1, kept1 = _round_ref(models, lists, alphas, tf1, compression or (0, 0, 0))
    got1 = pr.run().cpu().numpy()
    torch.cuda.synchronize()
    assert np.array_equal(got1, ref1), info
    if compression:
        assert pr.kept.cpu().tolist() == kept1, info
    # two chained rounds (the second mixes the first's output), replayed from a graph or eager
    ref2, _ = _round_ref(ref1, lists, alphas, tf1, compression or (0, 0, 0))
    pr2 = PopulationRound(gpu, torch.from_numpy(models).cuda())
    pr2.set_topology(lists, policy, use_window=use_window, numerics="tf1" if tf1 else "fp32",
                     compression=compression)
    got2 = pr2.rounds(2, graph=bool(rng.random() < 0.5)).cpu().numpy()
    assert np.array_equal(got2, ref2), info + ("rounds(2)",)
