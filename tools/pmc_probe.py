#!/usr/bin/env python3
"""Workload for one rocprofv3 PMC pass (run BY bench.py as a child process, under the profiler):
a few launches of the bench's dominant kernel (mix_vec_kernel through cfa_mix_seq_f32) on the
bench's bucket shape, K neighbour buckets + the local + the output, all resident in HBM.

Usage: rocprofv3 --pmc FETCH_SIZE -d DIR -o fetch --output-format csv -- \
           python tools/pmc_probe.py --params P --neighbours K [--launches 6]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, required=True)
    ap.add_argument("--neighbours", type=int, required=True)
    ap.add_argument("--launches", type=int, default=6)
    a = ap.parse_args()
    import torch
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    g = torch.Generator(device="cuda").manual_seed(20261015)
    rows = torch.empty((a.neighbours + 1, a.params), device="cuda")
    rows.normal_(generator=g)
    out = torch.empty(a.params, device="cuda")
    launch = eng.prepare_mix_seq(out, rows[0], list(rows[1:]), [1.0 / (a.neighbours + 1)] * a.neighbours)
    for _ in range(a.launches):
        launch()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
