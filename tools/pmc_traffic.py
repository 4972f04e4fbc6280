#!/usr/bin/env python3
"""Per-launch HBM traffic of the CFA mix kernel from rocprofv3 PMC passes.

Counters are collected in separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass
on gfx950, MI355X_MICROARCH.md §rocprofv3 PMC slots). Corrections per MI355X_MICROARCH.md §HBM:
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a
wide coalesced streaming read, so it is doubled. Writes profiles/<tag>_pmc_traffic.json.

Usage: tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv>
         --params P --neighbours K --out profiles/r01_pmc_traffic.json
"""
import argparse
import csv
import json
import statistics


def per_dispatch(path, counter, kernel_substr):
    vals = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") != counter or kernel_substr not in row.get("Kernel_Name", ""):
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", default="mix_vec_kernel")
    ap.add_argument("--params", type=int, required=True)
    ap.add_argument("--neighbours", type=int, required=True)
    ap.add_argument("--devices-per-launch", type=int, default=1,
                    help="window passes (cfa_mix_window_f32): devices mixed per launch")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch_csv, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write_csv, "WRITE_SIZE", a.kernel)
    if not fetch or not write:
        raise SystemExit("no dispatches of %s found" % a.kernel)
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    read_bytes = 2.0 * f_kib * 1024.0   # gfx950 FETCH_SIZE reads half of a wide coalesced stream
    write_bytes = w_kib * 1024.0
    B = a.devices_per_launch
    algorithmic = B * (a.neighbours + 2) * a.params * 4
    res = {
        "kernel": a.kernel, "params": a.params, "neighbours": a.neighbours, "devices_per_launch": B,
        "dispatches": {"fetch_pass": len(fetch), "write_pass": len(write)},
        "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib,
        "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count on 16B/lane streams); write = WRITE_SIZE x 1024",
        "hbm_read_bytes_per_launch": read_bytes, "hbm_write_bytes_per_launch": write_bytes,
        "hbm_bytes_per_launch": read_bytes + write_bytes,
        "algorithmic_bytes_per_launch": algorithmic,
        "traffic_over_algorithmic": (read_bytes + write_bytes) / algorithmic,
    }
    if B > 1:  # a window pass must read its B + K rows once and write B outputs
        res["window_min_bytes_per_launch"] = (2 * B + a.neighbours) * a.params * 4
        res["traffic_over_window_min"] = (read_bytes + write_bytes) / res["window_min_bytes_per_launch"]
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
