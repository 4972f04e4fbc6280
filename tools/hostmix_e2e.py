#!/usr/bin/env python3
"""End-to-end cost of the drop-in host path at the north-star size: K = 8 neighbour models of
P = 25M fp32 parameters held as pageable numpy arrays (per-layer, as the reference holds them),
mixed through HostMixer.mix (pack into pinned staging, H2D, kernel, D2H, unpack). Also times
the pack alone and torch's parallel copy into the same pinned buffer."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from federated_amd.consensus._runtime import mixer  # noqa: E402
from federated_amd.engine import BucketLayout  # noqa: E402

K = 8
shapes = [(5000, 4000), (4000,), (1000, 4996), (4,)]  # 25,000,000 params in 4 layers
rng = np.random.default_rng(0)
local = [rng.standard_normal(s, dtype=np.float32) for s in shapes]
nbrs = [[rng.standard_normal(s, dtype=np.float32) for s in shapes] for _ in range(K)]
P = sum(int(np.prod(s)) for s in shapes)
mx = mixer()
al = [1.0 / (K + 1)] * K


def med(fn, n=5):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


from federated_amd.consensus import _runtime as R  # noqa: E402

R.PIPELINE_ZERO_COPY = False
t_mix_copies = med(lambda: mx.mix(local, nbrs, al))
R.PIPELINE_ZERO_COPY = True
t_mix = med(lambda: mx.mix(local, nbrs, al))
lay = BucketLayout.of(local)
pinned = torch.empty((K + 1) * P, dtype=torch.float32, pin_memory=True)
hv = pinned.numpy().reshape(K + 1, P)


def pack_numpy():
    lay.pack(local, hv[0])
    for j in range(K):
        lay.pack(nbrs[j], hv[j + 1])


def pack_torch():
    for j, m in enumerate([local] + nbrs):
        for k, a in enumerate(m):
            b, e = lay.segment(k)
            pinned[j * P + b:j * P + e].copy_(torch.from_numpy(a).reshape(-1))


print(json.dumps({"P": P, "K": K, "hostmixer_mix_ms": round(t_mix * 1e3, 2),
                  "hostmixer_mix_ms_copy_pipeline": round(t_mix_copies * 1e3, 2),
                  "pack_numpy_ms": round(med(pack_numpy) * 1e3, 2), "pack_torch_ms": round(med(pack_torch) * 1e3, 2),
                  "torch_threads": torch.get_num_threads(), "bytes_packed": (K + 1) * P * 4}))
