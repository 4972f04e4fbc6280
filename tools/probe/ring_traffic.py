#!/usr/bin/env python3
"""HBM traffic of the bench's ring round at the per-rank shapes of N = 1, 2, 4, 8 (128 devices,
K = 8, every device's 1/N element slice), from rocprofv3 PMC passes over tools/pmc_probe.py --ring
(bench.live_traffic, as the N > 1 bench line measures it), against the algorithmic bytes.
GPU box: python tools/probe/ring_traffic.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

P, K, D = 25_000_000, 8, 128
for n in (8, 4, 2, 1):
    p = P // n
    live, note = bench.live_traffic(p, K, timeout=240, ring=D)
    alg = (K + 2) * p * 4
    print(json.dumps({"experiment": "tools/probe/ring_traffic.py", "n_gpus_shape": n, "params_per_rank": p,
                      "devices": D, "algorithmic_bytes_per_mix": alg,
                      "traffic_bytes_per_mix": round(live, 1) if live is not None else None,
                      "traffic_over_algorithmic": round(live / alg, 4) if live is not None else None,
                      "note": note}), flush=True)
