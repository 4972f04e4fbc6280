#!/usr/bin/env python3
"""Is the "placement level" of the streaming mix (the same K = 8 x 25M mix at
~150 / ~158 / ~162 / ~167 us) a property of the allocation, or of the chip's clocks and power
state at the time?

Allocates S separate (input, output) stack pairs, then for SECONDS round-robins over them: a
batch of REPS back-to-back production mixes on one pair (HIP events), then one read of the GPU's
own metrics through amdsmi (read-only: current memory / fabric / SoC / gfx clocks, socket power,
throttle status, HBM temperature). One JSON line per batch, then a summary: the batch times
grouped by pair and by each clock's value. If the levels follow the clocks across pairs, the
allocation is not what sets them.

Usage: python tools/probe/clock_levels.py [--seconds 40] [--pairs 3] [--reps 20]"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

KEYS = ("current_uclk", "current_fclk", "current_socclk", "current_gfxclk", "average_uclk_frequency",
        "average_fclk_frequency", "average_socclk_frequency", "average_gfxclk_frequency",
        "current_socket_power", "average_socket_power", "throttle_status", "indep_throttle_status",
        "temperature_mem", "temperature_hotspot", "average_umc_activity", "average_gfx_activity",
        "pcie_link_speed", "xgmi_link_speed")


def open_metrics():
    """A function returning the visible GPU's metrics dict, or None when amdsmi is unavailable."""
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        props = torch.cuda.get_device_properties(0)
        want = (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", None),
                getattr(props, "pci_device_id", None))
        handles = amdsmi.amdsmi_get_processor_handles()
        pick = None
        for h in handles:
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
            dom, bus, rest = bdf.split(":")
            if want[1] is not None and int(bus, 16) == want[1] and int(dom, 16) == want[0]:
                pick = h
        if pick is None:
            pick = handles[0] if len(handles) == 1 else None
        if pick is None:
            return None, f"no amdsmi handle matches the visible GPU {want} among {len(handles)}"
        return (lambda: amdsmi.amdsmi_get_gpu_metrics_info(pick)), None
    except Exception as exc:  # reported in the output
        return None, f"{type(exc).__name__}: {exc}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=40.0)
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--carve-gib", type=int, default=0,
                    help="carve each pair's input rows and output from allocations of this many GiB (as "
                         "placement.calibrated_stacks does); 0 = plain allocations of the exact size")
    a = ap.parse_args()
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    P, K = a.params, 8
    metrics, err = open_metrics()
    if metrics is not None:
        m0 = metrics()
        print(json.dumps({"metrics_keys": sorted(k for k, v in m0.items() if isinstance(v, (int, float)))}),
              flush=True)
    else:
        print(json.dumps({"metrics_error": err}), flush=True)
    pairs = []
    hold = []
    for s in range(a.pairs):
        if a.carve_gib:
            big_in = torch.empty(a.carve_gib << 28, device="cuda")  # GiB of fp32
            big_out = torch.empty(a.carve_gib << 28, device="cuda")
            hold += [big_in, big_out]
            ins = big_in[:(K + 1) * P].view(K + 1, P).normal_()
            out = big_out[:P]
        else:
            ins = torch.empty((K + 1, P), device="cuda").normal_()
            out = torch.empty(P, device="cuda")
        pairs.append((ins, out))
    alphas = [1.0 / (K + 1)] * K
    fns = [eng.prepare_mix_seq(out, ins[0], [ins[j] for j in range(1, K + 1)], alphas) for ins, out in pairs]
    rows = []
    t_end = time.time() + a.seconds
    i = 0
    while time.time() < t_end:
        s = i % len(pairs)
        fn = fns[s]
        for _ in range(3):
            fn(None)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(a.reps):
            fn(None)
        ev1.record()
        ev1.synchronize()
        us = ev0.elapsed_time(ev1) * 1e3 / a.reps
        row = {"batch": i, "pair": s, "mix_us": round(us, 2)}
        if metrics is not None:
            try:
                m = metrics()
                for k in KEYS:
                    v = m.get(k)
                    if isinstance(v, (int, float)):
                        row[k] = v
            except Exception as exc:
                row["metrics_error"] = str(exc)
        rows.append(row)
        print(json.dumps(row), flush=True)
        i += 1
    summary = {"by_pair": {}, "by_clock": {}}
    for s in range(len(pairs)):
        t = [r["mix_us"] for r in rows if r["pair"] == s]
        if t:
            summary["by_pair"][s] = {"n": len(t), "median_us": round(statistics.median(t), 2),
                                     "min_us": min(t), "max_us": max(t)}
    for k in ("current_uclk", "current_fclk", "current_socclk", "average_uclk_frequency",
              "average_fclk_frequency", "throttle_status"):
        groups = {}
        for r in rows:
            if k in r:
                groups.setdefault(r[k], []).append(r["mix_us"])
        if groups:
            summary["by_clock"][k] = {str(v): {"n": len(t), "median_us": round(statistics.median(t), 2)}
                                      for v, t in sorted(groups.items())}
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    main()
