#!/usr/bin/env python3
"""Workload for one rocprofv3 PMC pass (run BY bench.py as a child process, under the profiler):
a few launches of the bench's dominant kernel (mix_vec_kernel through cfa_mix_seq_f32) on the
bench's bucket shape, K neighbour buckets + the local + the output, all resident in HBM.

With --ring D: the bench's population round instead, D device mixes of a [D, P] stack, device i
with its K ring-window neighbours (K // 2 below, the rest above, wrapping), into a [D, P] output
stack. That is the N > 1 headline's per-rank shape (every device, a 1/N element slice), whose rows
are short enough that the window's rows can be re-read from the Infinity Cache.

Usage: rocprofv3 --pmc FETCH_SIZE -d DIR -o fetch --output-format csv -- \
           python tools/pmc_probe.py --params P --neighbours K [--launches 6] [--ring D]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, required=True)
    ap.add_argument("--neighbours", type=int, required=True)
    ap.add_argument("--launches", type=int, default=6)
    ap.add_argument("--ring", type=int, default=0, help="D: one population round of D ring-window mixes per launch count")
    a = ap.parse_args()
    import torch
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    g = torch.Generator(device="cuda").manual_seed(20261015)
    K = a.neighbours
    alphas = [1.0 / (K + 1)] * K
    if a.ring:
        D, hl = a.ring, K // 2
        if D < K + 1:
            raise SystemExit("--ring needs at least K + 1 devices")
        rows = torch.empty((D, a.params), device="cuda")
        rows.normal_(generator=g)
        outs = torch.empty((D, a.params), device="cuda")
        offs = [d for d in range(-hl, K - hl + 1) if d != 0]
        mixes = [eng.prepare_mix_seq(outs[i], rows[i], [rows[(i + d) % D] for d in offs], alphas) for i in range(D)]
        for _ in range(max(1, a.launches // 3)):  # rounds
            for m in mixes:
                m()
        torch.cuda.synchronize()
        return
    rows = torch.empty((a.neighbours + 1, a.params), device="cuda")
    rows.normal_(generator=g)
    out = torch.empty(a.params, device="cuda")
    launch = eng.prepare_mix_seq(out, rows[0], list(rows[1:]), alphas)
    for _ in range(a.launches):
        launch()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
