#!/usr/bin/env python3
"""Strong-scaling cost model of the bench's population round, computed from the
same RoutePlan the bench runs, so the table there can be regenerated:

  T(N) = max(L * t_mix * (1 + delta), C_halo / B_link + t_tail),   speed-up = T(1) / T(N)

L = devices per rank (x the element slice for params / hybrid), t_mix = one device mix on one
GPU (measured: 0.166 ms for K = 8 x 25M), C_halo = RoutePlan.critical_elems * 4 bytes (the sum
over groups of the busiest link's load), t_tail = the boundary devices of the last stage, B_link
= xGMI point-to-point rate per direction (an assumption: 50 and 64 GB/s by default), delta = the
mixes' slowdown while RCCL copies run (measured with a stand-in: 0.10-0.16). With ``--lane``
rates > 0 the halo may also take the host lane (federated_amd/hostlane.py: PCIe through pinned
host memory, that rate per GPU and direction): the plan is then ``halo.choose_route``'s pick at
those rates and C_halo / B_link becomes its predicted exchange time (for lane 0 the two agree).

Pure host arithmetic (no GPU). Usage: python tools/scale_model.py [--params P] [--devices D]

With ``--from-lines FILE`` (bench JSON lines, one per N, e.g. the driver's SCALE record or the
lines of `python bench.py --gpus N`), the model is re-evaluated with what each N > 1 line
MEASURED instead of the assumptions: B_link = the line's `config.links.median_GBps`, delta and
t_mix from its `decomposition`, T(1) from the N = 1 line's `ms_per_step`; each row prints the
model's speed-up next to the achieved one (value / value at N = 1)."""
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


def exchange_ms(world, partition, D, h, P, link_gbps, lane_gbps, groups=None):
    """The chosen plan's predicted exchange time at uniform link rates plus (lane_gbps > 0) the
    host lane's, and the MB it puts on the lane."""
    from federated_amd.halo import LANE_IN, LANE_OUT, choose_route
    from federated_amd.hostlane import DEFAULT_CHUNK_ELEMS, first_chunk_elems
    gd, gp = partition_shape(partition, world, D, groups)
    if gd < 2:
        return 0.0, 0.0
    tr = ring_transfers(gd, D // gd, h, h, P, slice_world=gp, slice_bounds=slice_bounds(P, gp))
    rates = {(a, b): link_gbps for a in range(world) for b in range(world) if a != b}
    if lane_gbps > 0:
        rates.update({(a, LANE_OUT): lane_gbps for a in range(world)})
        rates.update({(LANE_IN, a): lane_gbps for a in range(world)})
    fill = first_chunk_elems(DEFAULT_CHUNK_ELEMS) * 4
    plan, _ = choose_route(world, tr, rates_gbps=rates, lane_chunk_bytes=fill)
    return plan.predicted_ms(rates, lane_chunk_bytes=fill), plan.lane_elems() * 4 / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--devices", type=int, default=128)
    ap.add_argument("--half-window", type=int, default=4)
    ap.add_argument("--t-mix-ms", type=float, default=0.166, help="one K = 8 x 25M device mix on one GPU")
    ap.add_argument("--links", default="50,64", help="GB/s per xGMI link per direction (assumed)")
    ap.add_argument("--delta", default="0.10,0.16")
    ap.add_argument("--lane", default="0", help="GB/s of the host lane per GPU and direction (0 = xGMI only)")
    ap.add_argument("--from-lines", default=None,
                    help="bench JSON lines (one per N): re-evaluate the model with their measured link rate, "
                         "delta and t_mix and print it beside the achieved speed-up")
    a = ap.parse_args()
    if a.from_lines:
        return from_lines(a.from_lines)
    D, P, h = a.devices, a.params, a.half_window
    tmix = a.t_mix_ms * P / 25_000_000
    T1 = D * tmix
    links = [float(x) for x in a.links.split(",")]
    deltas = [float(x) for x in a.delta.split(",")]
    lanes = [float(x) for x in a.lane.split(",")]
    rows = [(2, "devices", None), (4, "devices", None), (4, "hybrid", 2), (8, "devices", None),
            (8, "hybrid", 4), (8, "hybrid", 2), (2, "params", None), (4, "params", None), (8, "params", None)]
    for N, part, g in rows:
        gd, gp = partition_shape(part, N, D, g)
        crit, relayed = critical_bytes(N, part, D, h, P, g)
        mixes = D // gd * tmix / gp
        out = {"N": N, "partition": part + (f" G={g}" if g else ""), "relayed": relayed,
               "mixes_per_rank_ms": round(mixes, 2), "critical_halo_MB": round(crit / 1e6, 1)}
        for bl in links:
            for ln in lanes:
                x_ms, lane_mb = (crit / (bl * 1e9) * 1e3, 0.0) if ln <= 0 else \
                    exchange_ms(N, part, D, h, P, bl, ln, g)
                tag = f"{bl:g}GBps" + (f",lane{ln:g}" if ln > 0 else "")
                if ln > 0:
                    out[f"lane_MB@{tag}"] = round(lane_mb, 1)
                for dl in deltas:
                    halo = x_ms + (2 * tmix / gp if crit else 0.0)
                    T = max(mixes * (1 + (dl if crit else 0.0)), halo)  # no exchange, no RCCL kernels
                    out[f"speedup@{tag},delta{dl:g}"] = round(T1 / T, 2)
        print(json.dumps(out))


def _lines(path):
    out = []
    with open(path) as fh:
        text = fh.read()
    try:  # a driver record: {"runs": [{"parsed": line}, ...]} or a list of lines
        doc = json.loads(text)
        items = doc if isinstance(doc, list) else doc.get("runs") or doc.get("results") or [doc]
        for it in items:
            line = it.get("parsed", it) if isinstance(it, dict) else None
            if isinstance(line, dict) and "n_gpus" in line:
                out.append(line)
    except ValueError:
        for raw in text.splitlines():
            raw = raw.strip()
            if raw.startswith("{"):
                line = json.loads(raw)
                if "n_gpus" in line:
                    out.append(line)
    return out


def from_lines(path):
    lines = sorted(_lines(path), key=lambda d: d["n_gpus"])
    one = next((d for d in lines if d["n_gpus"] == 1), None)
    if one is None:
        print(json.dumps({"error": f"no N = 1 line in {path}"}))
        return 1
    T1, v1 = one["ms_per_step"], one["value"]
    for d in lines:
        if d["n_gpus"] == 1:
            continue
        c, dc = d.get("config", {}), d.get("decomposition") or {}
        links = c.get("links") or {}
        row = {"N": d["n_gpus"], "partition": c.get("partition"), "achieved_speedup": round(d["value"] / v1, 2),
               "ms_per_step": d["ms_per_step"], "link_median_GBps": links.get("median_GBps"),
               "delta": dc.get("delta"), "t_mix_ms": dc.get("t_mix_ms"),
               "exchange_groups_ms": dc.get("exchange_groups_ms_sum")}
        if dc.get("model_prediction_ms"):
            row["model_ms"] = dc["model_prediction_ms"]
            row["model_speedup"] = round(T1 / dc["model_prediction_ms"], 2)
        route = c.get("halo_route") or {}
        if links.get("median_GBps") and route.get("critical_MB") and dc.get("t_mix_ms") is not None:
            L = c.get("devices_per_gpu") or 0
            pred = (route.get("autotune") or {}).get("predicted_ms")
            if route.get("lane") and pred:  # the kept plan's exchange at the probed link and lane rates
                halo = pred + dc.get("tail_ms", 0.0)
                row["host_lane_MB"] = route.get("lane_MB")
            else:
                halo = route["critical_MB"] * 1e6 / (links["median_GBps"] * 1e9) * 1e3 + dc.get("tail_ms", 0.0)
            comp = L * dc["t_mix_ms"] * (1 + max(0.0, dc.get("delta") or 0.0))
            row["probe_model_ms"] = round(max(comp, halo), 4)
            row["probe_model_speedup"] = round(T1 / max(comp, halo), 2)
        print(json.dumps(row))
    return 0


if __name__ == "__main__":
    sys.exit(main())
