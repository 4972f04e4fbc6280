#!/usr/bin/env python3
"""Exact optimum of the bench's staged ring-halo schedule, as a linear program (CPU, scipy).

The bench's `devices` partition at N ranks with a K = 2H ring window moves, in each of H stages,
one bucket row from every rank to each of its two ring neighbours (federated_amd/halo.py
ring_transfers). A row may go direct or through any third rank (two hops; the second hop lands in
the next group), and groups run back to back, so the exchange time is the sum over groups of the
busiest link's load. The LP splits every row continuously over its paths and minimises that sum:
a lower bound for any routing of this schedule, to compare with RoutePlan.critical_elems (the
integer greedy the bench runs). Prints one JSON line.

Usage: python tools/probe/halo_lp.py [--world 8] [--stages 4] [--row-mb 100]"""
import argparse
import json
import os
import sys

import numpy as np
from scipy.optimize import linprog

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def lp_optimum(N: int, S: int, row: float):
    flows = [(a, (a + 1) % N) for a in range(N)] + [(a, (a - 1) % N) for a in range(N)]
    paths = []  # (flow, first-group links, next-group links)
    for fi, (a, b) in enumerate(flows):
        paths.append((fi, [(a, b)], []))
        paths += [(fi, [(a, k)], [(k, b)]) for k in range(N) if k not in (a, b)]
    links = [(i, j) for i in range(N) for j in range(N) if i != j]
    P, G = len(paths), S + 1
    nv = S * P + G
    c = np.zeros(nv)
    c[S * P:] = 1.0
    A, bu = [], []
    for g in range(G):
        for l in links:
            row_ = np.zeros(nv)
            for s in (g, g - 1):
                if 0 <= s < S:
                    for pi, (_, h1, h2) in enumerate(paths):
                        if (s == g and l in h1) or (s == g - 1 and l in h2):
                            row_[s * P + pi] += 1.0
            row_[S * P + g] = -1.0
            A.append(row_)
            bu.append(0.0)
    Aeq, beq = [], []
    for s in range(S):
        for fi in range(len(flows)):
            row_ = np.zeros(nv)
            for pi, (f, _, _) in enumerate(paths):
                if f == fi:
                    row_[s * P + pi] = 1.0
            Aeq.append(row_)
            beq.append(row)
    r = linprog(c, A_ub=np.array(A), b_ub=bu, A_eq=np.array(Aeq), b_eq=beq, bounds=[(0, None)] * nv,
                method="highs")
    return float(r.fun), [float(x) for x in r.x[S * P:]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--stages", type=int, default=4)
    ap.add_argument("--row-mb", type=float, default=100.0)
    a = ap.parse_args()
    opt, groups = lp_optimum(a.world, a.stages, a.row_mb)
    from federated_amd.halo import RoutePlan, ring_transfers
    P = int(a.row_mb * 1e6 / 4)
    plan = RoutePlan(a.world, ring_transfers(a.world, 16, a.stages, a.stages, P), relay=True)
    got = plan.critical_elems() * 4 / 1e6
    print(json.dumps({"tool": "tools/probe/halo_lp.py", "world": a.world, "stages": a.stages, "row_MB": a.row_mb,
                      "lp_optimum_MB": round(opt, 2), "lp_group_max_MB": [round(x, 1) for x in groups],
                      "routeplan_critical_MB": round(got, 2), "routeplan_over_optimum": round(got / opt, 4),
                      "routeplan_units": plan.units}))


if __name__ == "__main__":
    main()
