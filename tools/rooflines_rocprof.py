#!/usr/bin/env python3
"""Join the event-timed roofline of every entry point (tools/kernel_rooflines.py, run under
`rocprofv3 --kernel-trace --stats`: `tools/gpu_session.sh TAG rlprof`) with the same run's
rocprofv3 kernel trace, so each row carries the kernel's average dispatch duration by rocprof
beside the HIP-event time and both fractions of the 8 TB/s peak.

  python tools/rooflines_rocprof.py ROOFLINES.log KERNEL_TRACE.csv > profiles/rNN_rooflines_rocprof.jsonl

The rocprof average covers every dispatch of the kernel in the run (the entry point's warm-up and
timed launches); the event time covers the timed launches only."""
import csv
import json
import statistics
import sys

PEAK = 8000.0
KERNEL = {  # entry point -> the kernel its 25M case launches (round-4/5 signatures)
    "cfa_mix_seq_f32": "mix_vec_kernel<8, 0, 2, 2>",
    "cfa_mix_seq_div_f32": "mix_vec_kernel<8, 2, 4, 1>",
    "cfa_mix_f32": "mix_vec_kernel<8, 1, 4, 1>",
    "cfa_mix_tf1_f32": "mix_tf1_vec_kernel<8, false, 0, 2>",
    "cfa_mix_tf1_wide_f32": "mix_tf1_vec_kernel<8, false, 2, 4>",
    "cfa_mix_seq_compress_f32": "mix_vec_compress_kernel<3, 2>",
    "cfa_compress_epilogue_f32": "compress_kernel<2>",
    "cfa_mewma_update_f32": "mewma_vec_kernel<2>",
    "cfa_mix_tf1_f64": "fold_f64_vec_kernel<4, 0, false>",
    "cfa_fold_f64": "fold_f64_vec_kernel<4, 2, false>",
    "cfa_mewma_tf1_f64": "mewma_tf1_f64_vec_kernel<2, false>",
    "cfa_mix_population_f32": "population_kernel<0>",
    "cfa_ge_population_step_f32": "ge_step_kernel(",
}


def main():
    log, trace = sys.argv[1], sys.argv[2]
    rows = []
    with open(log) as fh:
        for line in fh:
            line = line.strip()
            if line.startswith("{") and "kernel_entry" in line:
                rows.append(json.loads(line))
    with open(trace) as fh:
        disp = list(csv.DictReader(fh))
    for r in rows:
        pat = KERNEL.get(r["kernel_entry"])
        if pat is None:
            continue
        us = [(int(d["End_Timestamp"]) - int(d["Start_Timestamp"])) / 1e3 for d in disp if pat in d["Kernel_Name"]]
        names = {d["Kernel_Name"] for d in disp if pat in d["Kernel_Name"]}
        if not us:
            continue
        avg = statistics.mean(us)
        ev = r["avg_launch_ms"] * 1e3
        b = r["algorithmic_bytes"]
        print(json.dumps({"kernel_entry": r["kernel_entry"], "kernel": sorted(names)[0], "calls": len(us),
                          "rocprof_avg_us": round(avg, 2), "events_avg_us": round(ev, 1), "algorithmic_bytes": b,
                          "frac_events": round(b / (ev * 1e-6) / 1e9 / PEAK, 4),
                          "frac_rocprof": round(b / (avg * 1e-6) / 1e9 / PEAK, 4),
                          "note": "rocprof average over every dispatch of the kernel in the run (warm-up + timed); "
                                  "events over the timed launches"}))


if __name__ == "__main__":
    main()
