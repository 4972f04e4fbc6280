#!/usr/bin/env python3
"""(f3) CFA-GE neighbour-gradient evaluation latency at the driver's shapes
(federated_sample_CNN_CFA-GE.py / _2NN_CFA-GE.py: 24 samples per device, N = 2 neighbour
models): the HIP launch alone (HIP events; the drop-in's batch-split launch and the
one-workgroup-per-model launch), the host call
(upload, launch, download), torch autograd on the same GPU (vmap over the models), and the
oracle's numpy float64 evaluation on one core. Prints one JSON line per model kind.
Usage: python tools/f3_latency.py [--models 2] [--samples 24] [--reps 200]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def torch_cost(logits, y):
    pred = torch.softmax(logits, dim=1)
    return torch.mean(-torch.sum(y * torch.log(torch.clamp(pred, 1e-15, 0.99)), dim=1))


def torch_cnn(x, W1, b1, W2, b2, stride=5):
    h = F.conv1d(F.pad(x.unsqueeze(1), (7, 7)), W1.permute(2, 1, 0), b1, stride=stride)
    h = F.max_pool1d(F.pad(torch.relu(h), (1, 1), value=float("-inf")), kernel_size=stride, stride=stride)
    return h.permute(0, 2, 1).reshape(h.shape[0], -1) @ W2 + b2


def torch_2nn(x, W1, b1, W2, b2):
    return torch.relu(x @ W1 + b1) @ W2 + b2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", type=int, default=2)
    ap.add_argument("--samples", type=int, default=24)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    from torch.func import grad, vmap
    from federated_amd.consensus import _tf1_models as T
    from federated_amd.engine import get_engine
    from oracle import cfa_oracle as orc
    eng = get_engine(0)
    rng = np.random.default_rng(0)
    B, M = a.samples, a.models
    x = rng.standard_normal((B, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[rng.integers(0, 8, B)]
    for kind, shapes in (("cnn", [(16, 1, 8), (8,), (168, 8), (8,)]), ("2nn", [(512, 32), (32,), (32, 8), (8,)])):
        ml = 1 if kind == "cnn" else 2
        models = [[(rng.standard_normal(s) * 0.1).astype(np.float32) for s in shapes] for _ in range(M)]
        P = sum(int(np.prod(s)) for s in shapes)
        xt, yt = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        mt = torch.from_numpy(np.stack([np.concatenate([m.reshape(-1) for m in mm]) for mm in models])).cuda()
        gt = torch.empty_like(mt)
        unsplit = (lambda: eng.grad_cnn(xt, yt, mt, gt, 16, 8, 5)) if ml == 1 else (lambda: eng.grad_2nn(xt, yt, mt, gt, 32))
        # the drop-in's launch: population form with each model's batch split over workgroups
        geom = {"filter": 16, "number": 8, "stride": 5} if ml == 1 else {"intermediate_nodes": 32}
        mrow = torch.arange(M, dtype=torch.int32, device="cuda")
        drow = torch.zeros(M, dtype=torch.int32, device="cuda")
        ws = eng.grad_workspace(M, B, P)
        split = lambda: eng.grad_rows(ml, xt.view(1, B, -1), yt.view(1, B, -1), mt, mrow, drow, gt, geom, workspace=ws)

        def timed(launch):
            for _ in range(10):
                launch()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                launch()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / a.reps
        kernel_us, unsplit_us = timed(split), timed(unsplit)
        T.gradients_batched(ml, x, y, models, stride=5)
        t0 = time.perf_counter()
        for _ in range(a.reps // 4):
            T.gradients_batched(ml, x, y, models, stride=5)
        host_us = (time.perf_counter() - t0) / (a.reps // 4) * 1e6
        fwd = torch_cnn if ml == 1 else torch_2nn
        params = [torch.stack([torch.from_numpy(np.squeeze(m[k]) if k in (1, 3) else m[k]) for m in models]).cuda()
                  for k in range(4)]
        fn = vmap(grad(lambda W1, b1, W2, b2: torch_cost(fwd(xt, W1, b1, W2, b2), yt), argnums=(0, 1, 2, 3)))
        for _ in range(5):
            fn(*params)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps // 4):
            fn(*params)
        torch.cuda.synchronize()
        torch_us = (time.perf_counter() - t0) / (a.reps // 4) * 1e6
        ref = (lambda m: orc.tf1_cnn_grads(x, y, *m, stride=5)) if ml == 1 else (lambda m: orc.tf1_2nn_grads(x, y, *m))
        t0 = time.perf_counter()
        for _ in range(20):
            for m in models:
                ref(m)
        numpy_us = (time.perf_counter() - t0) / 20 * 1e6
        print(json.dumps({"model": kind, "params": P, "samples": B, "neighbour_models": M,
                          "hip_kernel_us": round(kernel_us, 2), "hip_kernel_unsplit_us": round(unsplit_us, 2),
                          "batch_splits": eng.grad_splits(M, B, P), "hip_host_call_us": round(host_us, 1),
                          "torch_autograd_vmap_gpu_us": round(torch_us, 1), "numpy_f64_1core_us": round(numpy_us, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
