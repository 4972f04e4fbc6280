"""Whole-run trajectories: R consensus rounds of a simulated population run two
ways must agree bit for bit at every round:

* the reference's way: every device calls the TF2 drop-in ``CFA_process.federated_weights_computing``
  (consensus_v3.py:73-159 / consensus_v4.py:176-217) through the file protocol, reading its
  neighbours' previous-round models from ``results/dump_train_model{k}.npy``;
* the device-resident way: one ``topology.PopulationRound`` launch per round over the [D, P]
  stack, with the same neighbour lists and eps policy (eps = 1/(n+1)).

The per-device drop-in is itself pinned to the reference's outputs (test_gpu_consensus_golden),
so this extends that parity from one call to whole multi-round runs.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# VGG-1-like layer list, scaled down (CIFAR-100 driver order: conv W, b, conv W, b, dense W, b)
SHAPES = [(3, 3, 3, 8), (8,), (3, 3, 8, 8), (8,), (128, 10), (10,)]


@pytest.fixture
def workdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("FEDERATED_AMD_PAUSE_SCALE", "0")
    os.makedirs("results")
    return tmp_path


def _obj(layers):
    a = np.empty(len(layers), dtype=object)
    for i, l in enumerate(layers):
        a[i] = l
    return a


@pytest.mark.parametrize("version,N,D", [("v3", 2, 8), ("v3", 4, 9), ("v4", 1, 8)])
def test_population_rounds_reproduce_dropin_trajectory(gpu, workdir, version, N, D):
    from federated_amd import topology as T
    if version == "v3":
        from federated_amd.consensus.consensus_v3 import CFA_process
        lists = T.kregular_v3(D, N)
    else:
        from federated_amd.consensus.consensus_v4 import CFA_process
        lists = T.ring_v4(D, N)
    rng = np.random.default_rng(D * 10 + N)
    models = [[rng.standard_normal(s).astype(np.float32) for s in SHAPES] for _ in range(D)]
    sizes = [int(np.prod(s)) for s in SHAPES]
    flat = np.stack([np.concatenate([a.reshape(-1) for a in m]) for m in models])
    pr = T.PopulationRound(gpu, torch.from_numpy(flat).cuda())
    pr.set_topology(lists, T.alphas_tf2, use_window=False)
    procs = [CFA_process(D, d, N) for d in range(D)]
    for rnd in range(3):
        # the reference way: every device publishes, then every device mixes its neighbours' files
        for d in range(D):
            np.save(f"results/dump_train_model{d}.npy", _obj(models[d]), allow_pickle=True)
            np.savez(f"results/dump_train_variables{d}.npz", frame_count=rnd, epoch_count=rnd,
                     training_end=False, loss=0.5)
        new = []
        for d in range(D):
            p = procs[d]
            p.update_local_model(_obj([a.copy() for a in models[d]]))
            nb = lists[d]
            if version == "v4" and N < 2:
                out = p.federated_weights_computing(nb[0], N, rnd, 0.5, 0, 30)
            else:
                out = p.federated_weights_computing(np.asarray(nb), N, rnd, 0.5, 0, 30)
            new.append([np.asarray(a, dtype=np.float32) for a in out])
        models = new
        # the device-resident way: one launch for the population
        out = pr.run()
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for d in range(D):
            ref = np.concatenate([a.reshape(-1) for a in models[d]])
            assert np.array_equal(got[d], ref), (version, rnd, d)
        pr.models.copy_(out)
    assert sum(sizes) == flat.shape[1]


TF1_SHAPES = [(16, 1, 8), (8,), (168, 8), (8,)]  # CFA-GE CNN bucket, P = 1 488 (cfa.py's tensors)


@pytest.mark.parametrize("D,N,eps", [(5, 2, 1.0), (8, 3, 0.7)])
def test_tf1_population_reproduces_dropin_trajectory(gpu, workdir, D, N, eps):
    """TF1 protocol (cfa.py:105-154): at epoch e every device mixes its epoch-e model with its
    neighbours' models published at epoch e-1, and the driver assigns the returned fp64 arrays
    to fp32 TF variables. Four epochs of per-device drop-in calls through the .mat protocol
    equal Tf1PopulationRound rounds (one cfa_mix_population_tf1_f32 launch each) bit for bit."""
    from federated_amd import topology as T
    from federated_amd.consensus.cfa import CFA_process
    rng = np.random.default_rng(D * 10 + N)
    sizes = [int(np.prod(s)) for s in TF1_SHAPES]
    flat = lambda m: np.concatenate([np.asarray(a, dtype=np.float32).reshape(-1) for a in m])
    split = lambda v: [v[o:o + n].reshape(s) for o, n, s in zip(np.cumsum([0] + sizes[:-1]), sizes, TF1_SHAPES)]
    m0 = [[(rng.standard_normal(s) * 0.1).astype(np.float32) for s in TF1_SHAPES] for _ in range(D)]
    m1 = [[(rng.standard_normal(s) * 0.1).astype(np.float32) for s in TF1_SHAPES] for _ in range(D)]  # after an SGD step
    procs = [CFA_process(True, D, d, N) for d in range(D)]
    for d in range(D):  # epoch 0 publishes
        W1, b1, W2, b2 = m0[d]
        procs[d].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps)
    pr = T.Tf1PopulationRound(gpu, D, sum(sizes))
    pr.set_topology(T.kregular_tf1(D, N), T.alphas_tf1_cfa(eps, N))
    pr.load(torch.from_numpy(np.stack([flat(m) for m in m1])).cuda(), torch.from_numpy(np.stack([flat(m) for m in m0])).cuda())
    models = m1
    for epoch in range(1, 5):
        new = []
        for d in range(D):
            W1, b1, W2, b2 = models[d]
            out = procs[d].getFederatedWeight(W1, W2, b1, b2, epoch, np.zeros(3), eps)
            new.append(split(flat([np.float32(a) if np.ndim(a) == 0 else np.asarray(a).astype(np.float32) for a in out])))
        models = new  # the driver's fp32 TF variables
        pr.round()
        torch.cuda.synchronize()
        got = pr.current.cpu().numpy()
        for d in range(D):
            assert np.array_equal(got[d], flat(models[d])), (epoch, d)


ONGRAPHS_SHAPES = [(3, 3, 1, 4), (4,), (4096, 6), (6,)]  # FL_CFA_CNN_tf2.py:56-65, P = 24 622


@pytest.mark.parametrize("mode", [2, 3])
def test_tf1_ongraphs_population_with_compression_reproduces_dropin(gpu, workdir, mode):
    """Config 2's protocol (FL_CFA_CNN_tf2.py:253-266): per epoch a cfa_ongraphs consensus_mode 1
    call mixes all neighbours' epoch e-1 files (alpha = eps/(1+n)) with the DPCM compression
    epilogue on W2, then a stop_consensus call with no neighbours publishes the fp32 result (its
    DPCM pass against itself changes no value). The published model is thus the post-mix one,
    so without SGD in between every device mixes the current models: three epochs of these
    per-device calls equal three PopulationRound(numerics="tf1", compression=...) rounds bit for
    bit, outputs and every device's counter_param. (The sparse modes 1/4 also re-compress at
    publish time, in fp32; a population round does not model that second pass.)"""
    from federated_amd import topology as T
    from federated_amd.consensus.cfa_ongraphs import CFA_process
    D, N, eps = 8, 3, 1.0
    rng = np.random.default_rng(40 + mode)
    sizes = [int(np.prod(s)) for s in ONGRAPHS_SHAPES]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    flat = lambda m: np.concatenate([np.asarray(a, dtype=np.float32).reshape(-1) for a in m])
    split = lambda v: [v[offs[k]:offs[k + 1]].reshape(s) for k, s in enumerate(ONGRAPHS_SHAPES)]
    scale = 1e-4 if mode == 2 else 1e-3  # weights near the mode's threshold (DPCM differences)
    models = [[(rng.standard_normal(s) * scale).astype(np.float32) for s in ONGRAPHS_SHAPES] for _ in range(D)]
    lists = T.kregular_tf1(D, N)
    procs = [CFA_process(True, D, d, N, 1, mode, 1) for d in range(D)]  # graph 1: the passed lists
    for d in range(D):
        W1, b1, W2, b2 = models[d]
        procs[d].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), eps, [], False)
    pop = torch.from_numpy(np.stack([flat(m) for m in models])).cuda()
    pr = T.PopulationRound(gpu, pop)
    pr.set_topology(lists, T.alphas_tf1_ongraphs(eps), numerics="tf1", compression=(mode, int(offs[2]), int(offs[3])))
    for epoch in range(1, 4):
        new, counts = [], []
        for d in range(D):
            W1, b1, W2, b2 = (np.array(a) for a in models[d])
            res = procs[d].getFederatedWeight(W1, W2, b1, b2, epoch, np.zeros(3), eps, list(lists[d]), False)
            counts.append(int(res[4]))
            nxt = split(flat(res[:4]))  # the driver's fp32 variables
            procs[d].getFederatedWeight(nxt[0], nxt[2], nxt[1], nxt[3], epoch, np.zeros(3), eps, [], True)
            new.append(nxt)
        models = new
        out = pr.run()
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for d in range(D):
            assert np.array_equal(got[d], flat(models[d])), (epoch, d)
        assert pr.kept.cpu().tolist() == counts, epoch
        assert 0 < sum(counts) < D * sizes[2]
        pop.copy_(out)
