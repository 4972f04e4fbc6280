#!/usr/bin/env python3
"""Strong-scaling cost model of the bench's population round, computed from the
same RoutePlan the bench runs, so the table there can be regenerated:

  T(N) = max(L * t_mix * (1 + delta), C_halo / B_link + t_tail),   speed-up = T(1) / T(N)

L = devices per rank (x the element slice for params / hybrid), t_mix = one device mix on one
GPU (measured: 0.166 ms for K = 8 x 25M), C_halo = RoutePlan.critical_elems * 4 bytes (the sum
over groups of the busiest link's load), t_tail = the boundary devices of the last stage, B_link
= xGMI point-to-point rate per direction (an assumption: 50 and 64 GB/s by default), delta = the
mixes' slowdown while RCCL copies run (measured with a stand-in: 0.10-0.16).

Pure host arithmetic (no GPU). Usage: python tools/scale_model.py [--params P] [--devices D]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from federated_amd.halo import RoutePlan, ring_transfers  # noqa: E402
from federated_amd.population import partition_shape, slice_bounds  # noqa: E402


def critical_bytes(world, partition, D, h, P, groups=None, relay=True):
    gd, gp = partition_shape(partition, world, D, groups)
    if gd < 2:
        return 0, False
    tr = ring_transfers(gd, D // gd, h, h, P, slice_world=gp, slice_bounds=slice_bounds(P, gp))
    plan = RoutePlan(world, tr, relay=relay)
    return plan.critical_elems() * 4, plan.relay


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--devices", type=int, default=128)
    ap.add_argument("--half-window", type=int, default=4)
    ap.add_argument("--t-mix-ms", type=float, default=0.166, help="one K = 8 x 25M device mix on one GPU")
    ap.add_argument("--links", default="50,64", help="GB/s per xGMI link per direction (assumed)")
    ap.add_argument("--delta", default="0.10,0.16")
    a = ap.parse_args()
    D, P, h = a.devices, a.params, a.half_window
    tmix = a.t_mix_ms * P / 25_000_000
    T1 = D * tmix
    links = [float(x) for x in a.links.split(",")]
    deltas = [float(x) for x in a.delta.split(",")]
    rows = [(2, "devices", None), (4, "devices", None), (4, "hybrid", 2), (8, "devices", None),
            (8, "hybrid", 4), (8, "hybrid", 2), (2, "params", None), (4, "params", None), (8, "params", None)]
    for N, part, g in rows:
        gd, gp = partition_shape(part, N, D, g)
        crit, relayed = critical_bytes(N, part, D, h, P, g)
        mixes = D // gd * tmix / gp
        out = {"N": N, "partition": part + (f" G={g}" if g else ""), "relayed": relayed,
               "mixes_per_rank_ms": round(mixes, 2), "critical_halo_MB": round(crit / 1e6, 1)}
        for bl in links:
            for dl in deltas:
                halo = crit / (bl * 1e9) * 1e3 + (2 * tmix / gp if crit else 0.0)
                T = max(mixes * (1 + (dl if crit else 0.0)), halo)  # no exchange, no RCCL kernels
                out[f"speedup@{bl:g}GBps,delta{dl:g}"] = round(T1 / T, 2)
        print(json.dumps(out))


if __name__ == "__main__":
    main()
