#!/usr/bin/env python3
"""Per-call cost of the TF2 drop-in (consensus_v3.federated_weights_computing) at config C4's
model (CIFAR-100 VGG-1, P = 1 071 748, K = 4 neighbours) and of the FedAvg parameter server
(parameter_server_v2, 8 active devices), with the protocol sleeps off (FEDERATED_AMD_PAUSE_SCALE=0):
the whole call, and its file loads alone, with libcfa's .npy/.npz reader (the default) and with
fresh read buffers, and with np.load in its place. Also the radar CNN (C5's TF2 shapes, P = 3 745 446).

Usage: python tools/probe/tf2_calls.py [--reps 30]"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

os.environ.setdefault("FEDERATED_AMD_PAUSE_SCALE", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from federated_amd import npyfile  # noqa: E402
from federated_amd.consensus import _ps, _runtime as R, _tf2, consensus_v3, parameter_server_v2  # noqa: E402

VGG1 = [(3, 3, 3, 32), (32,), (3, 3, 32, 32), (32,), (8192, 128), (128,), (128, 100), (100,)]
RADAR = [(8, 8, 1, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (7168, 512), (512,), (512, 6), (6,)]


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def weights(shapes, rng):
    w = np.empty(len(shapes), dtype=object)
    for i, s in enumerate(shapes):
        w[i] = rng.standard_normal(s).astype(np.float32)
    return w


MODES = {
    "native": None,                                                   # libcfa's reader, slot buffers
    "native_t4": None,                                                # the same, 4 pipeline copy threads
    "native_t1": None,                                                # the same, 1 pipeline copy thread
    "native_fresh": lambda p, slot=None: npyfile.load(p),             # libcfa's reader, fresh buffers
    "np_load": lambda p, slot=None: np.load(p, allow_pickle=True),    # the reference's loader
}


def interleaved(fns, reps, rounds=6):
    """Median over `rounds` interleaved passes of every mode (A B C A B C ...), each pass the
    median of reps // rounds calls: slow drifts of the host hit every mode alike."""
    acc = {m: {k: [] for k in fns} for m in MODES}
    for _ in range(rounds):
        for m in MODES:
            use_loader(m)
            for k, fn in fns.items():
                acc[m][k].append(med(fn, max(3, reps // rounds)))
    return {m: {k: round(statistics.median(v), 3) for k, v in d.items()} for m, d in acc.items()}


def use_loader(mode):
    """Swap the drop-in's loader (the modules call npyfile.load(path[, slot=...]))."""
    fn = MODES[mode]
    R.NATIVE_THREADS = {"native_t4": 4, "native_t1": 1}.get(mode, 0)
    for mod in (_tf2, _ps, parameter_server_v2):
        mod.npyfile = npyfile if fn is None else type("L", (), {"load": staticmethod(fn)})


def tf2_call(shapes, K, reps):
    rng = np.random.default_rng(0)
    devices = K + 1
    for k in range(devices):
        np.savez(f"results/dump_train_variables{k}.npz", frame_count=100, epoch_loss_history=[0.5],
                 training_end=False, epoch_count=5, loss=0.25)
        np.save(f"results/dump_train_model{k}.npy", weights(shapes, rng), allow_pickle=True)
    p = consensus_v3.CFA_process(devices, 0, K)
    local = weights(shapes, rng)
    nbrs = list(range(1, K + 1))

    def call():
        p.update_local_model(local.copy())
        p.federated_weights_computing(nbrs, K, 5, 0.5)

    def loads():
        for k in nbrs:
            d = _tf2.npyfile.load(f"results/dump_train_variables{k}.npz")
            d["epoch_count"], d["training_end"]
            _tf2.npyfile.load(f"results/dump_train_model{k}.npy", slot=("tf2", k))
    out = interleaved({"call_ms": call, "loads_ms": loads}, reps)
    use_loader("native")
    p.update_local_model(local.copy())
    p.federated_weights_computing(nbrs, K, 5, 0.5)
    assert p.local_weights[0] is not local[0]  # the mix ran (a failed load would skip it)
    return out


def ps_call(shapes, devices, reps):
    rng = np.random.default_rng(1)
    for k in range(devices):
        np.savez(f"results/dump_train_variables{k}.npz", frame_count=100, epoch_loss_history=[0.5],
                 training_end=False, epoch_count=5, loss=0.25)
        np.save(f"results/dump_train_model{k}.npy", weights(shapes, rng), allow_pickle=True)
    indexes_tx = np.tile(np.arange(devices)[:, None], (1, 4))
    ps = parameter_server_v2.Parameter_Server(devices, weights(shapes, rng), devices, indexes_tx)

    def call():
        ps.federated_target_weights_aggregation(1, aggregation_type=0)
    out = interleaved({"call_ms": call}, reps)
    use_loader("native")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=60)
    a = ap.parse_args()
    old = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        os.makedirs("results")
        try:
            rows = [
                {"case": "C4 TF2 consensus_v3, VGG-1 P=1071748, K=4", **tf2_call(VGG1, 4, a.reps)},
                {"case": "TF2 consensus_v3, radar CNN P=3745446, K=2", **tf2_call(RADAR, 2, a.reps)},
                {"case": "parameter_server_v2 FedAvg, VGG-1, 8 active devices", **ps_call(VGG1, 8, a.reps)},
            ]
        finally:
            os.chdir(old)
    for r in rows:
        print(json.dumps({"experiment": "tools/probe/tf2_calls.py", **r}), flush=True)


if __name__ == "__main__":
    main()
