#!/usr/bin/env python3
"""Measurements at the functional BASELINE configs (the bench line is the 8 x 25M headline;
these are the reference's own shapes). Prints one JSON line per config.

configs[0..2] (one device's consensus call, files and protocol included, protocol sleeps off):
    drop-in call latency (median of repeated calls) and the numpy restatement of the same
    arithmetic (oracle, CPU) for context.
configs[3..4] (whole population round, buckets resident in HBM): one population-kernel launch
    (cfa_mix_population_f32) per round; algorithmic GB/s; numpy per-device loop on one core.
"""
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["FEDERATED_AMD_PAUSE_SCALE"] = "0"

import numpy as np  # noqa: E402
import scipy.io as sio  # noqa: E402
import torch  # noqa: E402

from federated_amd import matfile, topology as T  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402
from oracle import cfa_oracle as O  # noqa: E402


def med_time(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def tf1_call(shapes, K, N, module, reps=20, **kw):
    from federated_amd.consensus import cfa, cfa_ongraphs
    rng = np.random.default_rng(0)
    models = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(K)]
    old = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            if module == "cfa":
                procs = [cfa.CFA_process(True, K, j, N) for j in range(K)]
                for j in range(K):
                    W1, b1, W2, b2 = models[j]
                    procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), 1.0)
                p = procs[1]
                W1, b1, W2, b2 = models[1]
                call = lambda: p.getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), 1.0)
                nbr = p.neighbor_vec
            else:
                procs = [cfa_ongraphs.CFA_process(True, K, j, N, 6, kw["compression"], 1) for j in range(K)]
                for j in range(K):
                    W1, b1, W2, b2 = models[j]
                    procs[j].getFederatedWeight(W1, W2, b1, b2, 0, np.zeros(3), 1.0, [], False)
                p = procs[1]
                nbr = [0, 2, 3][:N]
                W1, b1, W2, b2 = models[1]
                call = lambda: p.getFederatedWeight(W1, W2, b1, b2, 1, np.zeros(3), 1.0, nbr, False)
            call()
            t_call = med_time(call, reps)
            local = models[1]
            nbrs = [models[int(j)] for j in nbr]
            wf = [O.tf1_weight_factor(K, 1, int(j), (N - 1) if module == "cfa" else len(nbr)) for j in nbr]

            def numpy_path():
                out = O.tf1_mix(local, nbrs, 1.0, wf)
                if module != "cfa" and kw["compression"]:
                    O.tf1_compress(np.asarray(out[2], dtype=np.float64), local[2], kw["compression"])
            t_np = med_time(numpy_path, reps)
            t_io = med_time(lambda: [matfile.loadmat(f"datamat{int(j)}_0.mat") for j in nbr], reps)
            t_io_scipy = med_time(lambda: [sio.loadmat(f"datamat{int(j)}_0.mat") for j in nbr], reps)
            save = {"weights1": local[0], "biases1": local[1], "weights2": local[2], "biases2": local[3],
                    "epoch": 1, "loss_sample": np.zeros(3), "counter_param": 1}
            t_save = med_time(lambda: matfile.savemat("bench_save.mat", save), reps)
            t_save_scipy = med_time(lambda: sio.savemat("bench_save.mat", save), reps)
        finally:
            os.chdir(old)
    P = sum(int(np.prod(s)) for s in shapes)
    return {"P": P, "neighbours": len(nbr), "dropin_call_ms": round(t_call * 1e3, 3),
            "of_which_mat_loads_ms": round(t_io * 1e3, 3), "scipy_loadmat_ms": round(t_io_scipy * 1e3, 3),
            "of_which_mat_save_ms": round(t_save * 1e3, 3), "scipy_savemat_ms": round(t_save_scipy * 1e3, 3),
            "numpy_arith_ms": round(t_np * 1e3, 3)}


def population(D, P, lists, policy, reps=20, use_window=None):
    eng = get_engine(0)
    models = torch.randn(D, P, device="cuda")
    pr = T.PopulationRound(eng, models)
    pr.set_topology(lists, policy, use_window)
    pr.run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pr.run()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    # R rounds replayed from captured hipGraphs (PopulationRound.rounds): kernels only, no
    # per-round Python launch path (the eager loop above also pays no copy: it re-mixes models)
    R = 10 * reps
    pr.rounds(R)
    torch.cuda.synchronize()
    e0.record()
    pr.rounds(R)
    e1.record()
    torch.cuda.synchronize()
    t_graph = e0.elapsed_time(e1) / R * 1e-3
    B = sum((len(l) + 2) * P * 4 for l in lists)
    host = models.cpu().numpy()

    def numpy_round():
        for d in range(D):
            O.sequential_mix(host[d], [host[j] for j in lists[d]], policy(lists[d], d, D))
    t_np = med_time(numpy_round, 2)
    return {"devices": D, "P": P, "path": "window" if pr.window else "csr", "round_us": round(t * 1e6, 1),
            "GBps": round(B / t / 1e9, 1), "round_us_graph": round(t_graph * 1e6, 2),
            "GBps_graph": round(B / t_graph / 1e9, 1),
            "numpy_round_ms_1core": round(t_np * 1e3, 2), "speedup_vs_numpy": round(t_np / t, 1)}


def tf1_population(D, P, N, eps, rounds=200, compression=None):
    """A TF1 population resident on the GPU against the numpy fp64 chain per device on one core:
    cfa.py (topology.Tf1PopulationRound: neighbours at epoch e-1), or with ``compression=(mode,
    cbegin, cend)`` cfa_ongraphs mode 1 (PopulationRound(numerics="tf1"): alpha eps/(1+n), the
    compression epilogue; numpy: oracle.tf1_compress on the W2 segment). One launch per round,
    fp64 chain rounded once."""
    eng = get_engine(0)
    lists = T.kregular_tf1(D, N)
    cur = torch.randn(D, P, device="cuda")
    if compression:
        # cfa_ongraphs mode 1 publishes the post-mix model: neighbours are the current models
        pol = T.alphas_tf1_ongraphs(eps)
        pr = T.PopulationRound(eng, cur)
        pr.set_topology(lists, pol, numerics="tf1", compression=compression)
        pr.round, pr.previous = pr.run, cur
    else:
        pol = T.alphas_tf1_cfa(eps, N)
        pr = T.Tf1PopulationRound(eng, D, P)
        pr.set_topology(lists, pol)
        pr.load(cur, torch.randn(D, P, device="cuda"))
    for _ in range(5):
        pr.round()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(rounds):
        pr.round()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / rounds * 1e-3
    pr.rounds(3 * rounds)
    torch.cuda.synchronize()
    e0.record()
    pr.rounds(3 * rounds)
    e1.record()
    torch.cuda.synchronize()
    t_graph = e0.elapsed_time(e1) / (3 * rounds) * 1e-3
    hc, hp = cur.cpu().numpy(), pr.previous.cpu().numpy()

    def numpy_round():
        for d in range(D):
            w = O.tf1_mix_flat(hc[d], [hp[j] for j in lists[d]], pol(lists[d], d, D))
            if compression:
                mode, cb, ce = compression
                O.tf1_compress(np.array(w[cb:ce]), hc[d][cb:ce], mode)
    t_np = med_time(numpy_round, 3)
    return {"devices": D, "P": P, "neighbours": N, "round_us": round(t * 1e6, 1),
            "round_us_graph": round(t_graph * 1e6, 2), "numpy_fp64_round_ms_1core": round(t_np * 1e3, 3),
            "speedup_vs_numpy_graph": round(t_np / t_graph, 1)}


def _cpu_worker(args):
    seed, P, K, reps = args
    rng = np.random.default_rng(seed)
    local = rng.standard_normal(P, dtype=np.float32)
    nbrs = [rng.standard_normal(P, dtype=np.float32) for _ in range(K)]
    a = [1.0 / (K + 1)] * K
    t0 = time.perf_counter()
    for _ in range(reps):
        O.sequential_mix(local, nbrs, a)
    return time.perf_counter() - t0


def cpu_pool_round(P=25_000_000, K=8, workers=None, reps=3):
    """SURVEY §8d CPU baseline (2): one process per simulated device (the reference's process
    model, FL_CFA_CNN_tf2.py:317-319), `workers` devices mixing concurrently."""
    import multiprocessing as mp
    workers = workers or min(16, os.cpu_count() or 1)
    with mp.get_context("spawn").Pool(workers) as pool:
        t0 = time.perf_counter()
        times = pool.map(_cpu_worker, [(i, P, K, reps) for i in range(workers)])
        wall = time.perf_counter() - t0
    mix_time = max(times)  # the mixing phase (data generation excluded)
    return {"workers": workers, "P": P, "K": K, "mixes": workers * reps,
            "aggregate_GBps": round(workers * reps * (K + 2) * P * 4 / mix_time / 1e9, 2), "wall_s": round(wall, 1)}


def cfa_ge_population(D=16, N=2, B=24, ml=1, rounds=50):
    """Config 3 as a device-resident population (federated_amd.cfa_ge_population): one fast
    CFA-GE round for all D devices = one stage-1 population launch, one gradient launch for all
    D*N (device, neighbour) pairs, D MEWMA launches; against the oracle's float64 round on one
    core (the repo's numpy path: per-device mix, gradients and MEWMA)."""
    from federated_amd.cfa_ge_population import CfaGePopulation
    eng = get_engine(0)
    geom = ({"filter": 16, "number": 8, "stride": 5} if ml == 1 else {"intermediate_nodes": 32})
    full = {**geom, "input_data": 512, "classes": 8}
    rng = np.random.default_rng(3)
    lists = T.kregular_tf1(D, N)
    shapes = O.tf1_flat_shapes(ml, full)
    P = sum(int(np.prod(s)) for s in shapes)
    x = rng.standard_normal((D, B, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[rng.integers(0, 8, (D, B))]
    pop = CfaGePopulation(eng, ml, geom, torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), lists, 1.0, N,
                          0.99, 0.1, 0.1)
    W = (rng.standard_normal((D, P)) * 0.1).astype(np.float32)
    pop.load(torch.from_numpy(W).cuda(), torch.from_numpy(W).cuda())
    for _ in range(5):
        pop.round()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(rounds):
        pop.round()
    e1.record()
    torch.cuda.synchronize()
    host_us = (time.perf_counter() - t0) / rounds * 1e6
    gpu_us = e0.elapsed_time(e1) / rounds * 1e3
    # the same rounds replayed from captured 6-round hipGraphs (CfaGePopulation.rounds)
    R = 48 * 10
    pop.rounds(R)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    pop.rounds(R)
    e1.record()
    torch.cuda.synchronize()
    graph_host_us = (time.perf_counter() - t0) / R * 1e6
    graph_us = e0.elapsed_time(e1) / R * 1e3
    Nm = max(len(l) for l in lists)
    Wd = W.astype(np.float64)
    G = np.zeros((D, Nm, P))
    S = np.zeros((D, Nm, P))
    t = med_time(lambda: O.cfa_ge_population_round(Wd, Wd, G, S, lists, x, y, ml, full, 1.0, N, 0.99, 0.1, 0.1), 3)
    return {"devices": D, "neighbours": N, "samples": B, "P": P, "model": "cnn" if ml == 1 else "2nn",
            "round_us_gpu_events": round(gpu_us, 1), "round_us_host": round(host_us, 1),
            "round_us_graph": round(graph_us, 2), "round_us_graph_host": round(graph_host_us, 2),
            "numpy_round_ms_1core": round(t * 1e3, 2), "speedup_vs_numpy": round(t * 1e6 / host_us, 1),
            "speedup_vs_numpy_graph": round(t * 1e6 / graph_host_us, 1)}


def main():
    rows = []
    if len(sys.argv) > 1 and sys.argv[1] == "c3":
        rows.append({"config": "C3 CFA-GE CNN, 16 devices, N=2, device-resident population round",
                     **cfa_ge_population()})
        rows.append({"config": "C3 shapes with the 2NN model, 16 devices, N=2, device-resident population round",
                     **cfa_ge_population(ml=2)})
        for r in rows:
            print(json.dumps(r), flush=True)
        return
    dropin_only = len(sys.argv) > 1 and sys.argv[1] == "dropin"
    if not dropin_only:
        rows.append({"config": "CPU pool baseline: 8 x 25M mix, one process per device", **cpu_pool_round()})
    rows.append({"config": "C1 2NN, 4 devices, cfa.py (federated_sample_2NN_CFA.py)",
                 **tf1_call([(512, 32), (32,), (32, 8), (8,)], 4, 2, "cfa")})
    rows.append({"config": "C2 CNN FL_CFA_CNN_tf2 shapes, 8 devices, K=3, cfa_ongraphs mode 1, compression 2",
                 **tf1_call([(3, 3, 1, 4), (4,), (4096, 6), (6,)], 8, 3, "ongraphs", compression=2)})
    rows.append({"config": "C3 CFA-GE CNN, 16 devices, N=2 (stage-1 mix via cfa.py math)",
                 **tf1_call([(16, 1, 8), (8,), (168, 8), (8,)], 16, 2, "cfa")})
    if dropin_only:
        for r in rows:
            print(json.dumps(r), flush=True)
        return
    rows.append({"config": "C1 shapes as a device-resident TF1 population (Tf1PopulationRound), 4 devices, N=2",
                 **tf1_population(4, 16_680, 2, 1.0)})
    rows.append({"config": "C3 topology as a device-resident TF1 population (stage-1 mix only), 16 devices, N=2",
                 **tf1_population(16, 1_488, 2, 1.0)})
    rows.append({"config": "C2 as a device-resident TF1 population: FL_CFA_CNN_tf2 buckets, 8 devices, K=3, "
                           "cfa_ongraphs mode 1 alpha, compression 2 on W2",
                 **tf1_population(8, 24_622, 3, 1.0, compression=(2, 40, 40 + 4096 * 6))})
    rows.append({"config": "C4 CIFAR-100 VGG-1, 32 devices, K=4 window, one population launch",
                 **population(32, 1_071_748, [[(d + o) % 32 for o in (-2, -1, 1, 2)] for d in range(32)], T.alphas_tf2)})
    rows.append({"config": "C5 radar CNN, 128 devices, ring (v4 N=1), one population launch",
                 **population(128, 24_622, T.ring_v4(128, 1), T.alphas_tf2)})
    rows.append({"config": "C5 at 25M params/device (scaling shape), 32 devices ring (auto: window passes)",
                 **population(32, 25_000_000, T.ring_v4(32, 1), T.alphas_tf2, reps=5)})
    rows.append({"config": "C5 at 25M params/device, 32 devices ring, CSR population kernel",
                 **population(32, 25_000_000, T.ring_v4(32, 1), T.alphas_tf2, reps=5, use_window=False)})
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
