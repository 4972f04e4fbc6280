#!/usr/bin/env python3
"""Tf1PopulationRound with plain vs placement-calibrated stacks (federated_amd/placement.py,
``calibrated_rotation``) at a stack of 1 GiB or more: D = 64 devices, P = 4.2M, 4 random
neighbours each, the TF1 cfa_ongraphs policy. Each configuration runs in its own process (the
placement level is a property of a process's allocations), alternating, twice each.

Prints one JSON line per run: ms per round (HIP events over 10 rounds after 3 warm-up rounds) and
the algorithmic GB/s (sum over devices of (n + 2) * P * 4 bytes per round).
Usage: python tools/tf1_population_placement.py [--reps 2]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(mode: str, D: int, P: int, K: int, rounds: int) -> None:
    import numpy as np
    import torch
    from federated_amd import topology as T
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    pop = T.Tf1PopulationRound(eng, D, P, placement_candidates=6 if mode == "placed" else 0)
    rng = np.random.default_rng(7)
    lists = [[int(j) for j in rng.choice([k for k in range(D) if k != d], K, replace=False)] for d in range(D)]
    pop.set_topology(lists, T.alphas_tf1_ongraphs(1.0))
    g = torch.Generator(device="cuda").manual_seed(3)
    pop.current.normal_(generator=g)
    pop.previous.normal_(generator=g)
    for _ in range(3):
        pop.round()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(rounds):
        pop.round()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / rounds
    nbytes = sum(len(l) + 2 for l in lists) * P * 4
    print(json.dumps({"mode": mode, "D": D, "P": P, "K": K, "ms_per_round": round(ms, 4),
                      "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "frac": round(nbytes / (ms * 1e-3) / 8e12, 4),
                      "stack_GiB": round(D * P * 4 / 2 ** 30, 3), "placement": pop.placement}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", default=None)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--devices", type=int, default=64)
    ap.add_argument("--params", type=int, default=4_200_000)
    ap.add_argument("--neighbours", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=10)
    a = ap.parse_args()
    if a.child:
        child(a.child, a.devices, a.params, a.neighbours, a.rounds)
        return
    for _ in range(a.reps):
        for mode in ("plain", "placed"):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode, "--devices", str(a.devices),
                                "--params", str(a.params), "--neighbours", str(a.neighbours), "--rounds", str(a.rounds)],
                               timeout=300)
            if r.returncode != 0:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
