#!/usr/bin/env python3
"""Per-call latency of the drop-in host path against the numpy arithmetic it replaces, on the
same box in the same run (medians over 300 calls).

Shapes:
- C1, TF1 2NN (federated_sample_2NN_CFA.py, P = 16 680, 2 neighbours): HostMixer.mix_tf1 (the
  TF1 rule on the reference's dtypes, what cfa.py calls) and HostMixer.mix (the TF2 fp32 rule);
- C2, FL_CFA_CNN_tf2 (P = 24 622, 3 neighbours, compression mode 2 on W2): HostMixer.mix_tf1
  with the fused epilogue (what cfa_ongraphs.py calls).

Beside each: the oracle's numpy restatement of the same arithmetic (oracle.tf1_mix /
sequential_mix / tf1_compress, the reference's own expressions), and, for context, the bare
kernel on device-resident buckets with its stream synchronisation, and a synchronisation alone.
Usage: python tools/dropin_latency.py [--zero-copy-off] [--signal-off]
(--signal-off: end each zero-copy call with hipStreamSynchronize instead of the signal word)"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from federated_amd.consensus import _runtime as R  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402
from oracle import cfa_oracle as O  # noqa: E402

if "--zero-copy-off" in sys.argv:
    R.SINGLE_ZERO_COPY = R.TF1_ZERO_COPY = False
if "--signal-off" in sys.argv:
    R.SIGNAL_COMPLETION = False


def med(fn, n=300):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


rng = np.random.default_rng(0)
mx = R.mixer()
eng = get_engine(0)
res = {"experiment": "tools/dropin_latency.py", "zero_copy": R.SINGLE_ZERO_COPY and R.TF1_ZERO_COPY,
       "signal_completion": R.SIGNAL_COMPLETION}

# C1: 2NN shapes, 2 neighbours, eps = 1, N = 2 -> alpha = eps * wf = 1/2 each (cfa.py:66-76)
shapes = [(512, 32), (32,), (32, 8), (8,)]
local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(2)]
P = sum(int(np.prod(s)) for s in shapes)
al = [0.5, 0.5]
res["C1"] = {
    "P": P, "n": 2,
    "mix_tf1_us": med(lambda: mx.mix_tf1(local, nbrs, al)),
    "numpy_tf1_us": med(lambda: O.tf1_mix(local, nbrs, 1.0, [np.float64(a) for a in al])),
    "mix_fp32_us": med(lambda: mx.mix(local, nbrs, al)),
    "numpy_fp32_us": med(lambda: [O.sequential_mix(local[k], [x[k] for x in nbrs], al) for k in range(4)]),
}

# C2: FL_CFA_CNN_tf2 shapes, 3 neighbours, compression mode 2 on W2 (layer 2)
shapes2 = [(3, 3, 1, 4), (4,), (4096, 6), (6,)]
local2 = [(rng.standard_normal(s) * 1e-3).astype(np.float32) for s in shapes2]
nbrs2 = [[(rng.standard_normal(s) * 1e-3).astype(np.float32) for s in shapes2] for _ in range(3)]
al2 = [0.25, 0.25, 0.25]


def numpy_c2():
    out = O.tf1_mix(local2, nbrs2, 1.0, [np.float64(a) for a in al2])
    O.tf1_compress(np.asarray(out[2], dtype=np.float64), local2[2], 2)


res["C2"] = {
    "P": sum(int(np.prod(s)) for s in shapes2), "n": 3, "compression": 2,
    "mix_tf1_compress_us": med(lambda: mx.mix_tf1(local2, nbrs2, al2, compress=(2, 2))),
    "numpy_tf1_compress_us": med(numpy_c2),
}

d = [torch.randn(P, device="cuda") for _ in range(3)]
out = torch.empty(P, device="cuda")
launch = eng.prepare_mix_seq(out, d[0], d[1:], al)


def kernel_only():
    launch()
    torch.cuda.synchronize()


res["context"] = {"kernel_plus_sync_us": med(kernel_only), "sync_only_us": med(torch.cuda.synchronize)}
print(json.dumps(res))
