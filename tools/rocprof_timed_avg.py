#!/usr/bin/env python3
"""Average duration of a kernel's LAST n dispatches in a rocprofv3 kernel trace.

The bench launches the mix kernel outside its timed region too (the placement probe and its
settle loop, the warm-up rounds), so the --stats average over every dispatch mixes those in. The
timed region is the last `--steps` rounds, i.e. the last steps x launches-per-round dispatches:
this averages exactly those, for comparison with the bench line's HIP-event figure.

  python tools/rocprof_timed_avg.py TRACE.csv --last 2560 [--kernel "mix_vec_kernel<8, 0, 2, 2>"]
(kernel names before the round-3 store-policy split read "mix_vec_kernel<8, 0, 2, true>")
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, required=True)
    ap.add_argument("--kernel", default="mix_vec_kernel<8, 0, 2, 2>")
    a = ap.parse_args()
    with open(a.trace) as fh:
        rows = [r for r in csv.DictReader(fh) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    last = us[-a.last:]
    print(json.dumps({"kernel": a.kernel, "dispatches": len(us), "all_avg_us": round(statistics.mean(us), 3),
                      "last": len(last), "last_avg_us": round(statistics.mean(last), 3),
                      "last_median_us": round(statistics.median(last), 3)}))


if __name__ == "__main__":
    main()
