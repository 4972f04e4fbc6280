#!/usr/bin/env python3
"""Counter evidence for the streaming kernels below the headline's roofline fraction.

For each kernel: a child process launches it on HBM-resident buckets of the roofline shape
(tools/kernel_rooflines.py: P = 25M, the same fan-ins), and rocprofv3 collects, in passes of their
own (MI355X_MICROARCH.md §rocprofv3 PMC slots):
  1. FETCH_SIZE                      (TCC; KiB; gfx950 counts half of a 16-B/lane stream: x2)
  2. WRITE_SIZE                      (TCC; KiB)
  3. SQ_WAVES, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAIT_ANY,
     SQ_ACTIVE_INST_ANY, SQ_INSTS_VMEM_RD (8 SQ) + GRBM_GUI_ACTIVE, GRBM_COUNT (2 GRBM)
Per kernel it reports HBM bytes per launch against the algorithmic bytes (traffic ratio: above
1.0 = wasted re-reads), the share of wave time spent issuing VALU (SQ_ACTIVE_INST_VALU /
SQ_WAVE_CYCLES) and parked on memory (SQ_WAIT_ANY / SQ_WAVE_CYCLES), VALU instructions per
64 elements, and GRBM busy cycles per XCD. Rates come from tools/kernel_rooflines.py: launches timed
while counters are collected are not representative. The headline mix (cfa_mix_seq_f32, n = 8)
is the calibration row: its traffic ratio is 1.0001x (profiles/r01_pmc_traffic.json).

Usage: python tools/pmc_rows.py [--kernels a,b] [--out DIR]   (on the GPU box)
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
P_DEFAULT = 25_000_000

# name -> (entry point, algorithmic bytes per launch as a function of P, elements per launch)
ROWS = {
    "mix_seq_n8": ("cfa_mix_seq_f32", lambda P: 10 * P * 4, lambda P: P),
    "mix_seq_div_n8": ("cfa_mix_seq_div_f32", lambda P: 10 * P * 4, lambda P: P),
    "compress_epilogue_mode2": ("cfa_compress_epilogue_f32", lambda P: 3 * P * 4, lambda P: P),
    "fold_f64_div_n4": ("cfa_fold_f64", lambda P: 6 * P * 8, lambda P: P),
    "mewma_tf1_f64_n2": ("cfa_mewma_tf1_f64", lambda P: 8 * P * 8, lambda P: P),
    "mix_tf1_n8": ("cfa_mix_tf1_f32", lambda P: 10 * P * 4, lambda P: P),
    "mix_tf1_wide_n8": ("cfa_mix_tf1_wide_f32", lambda P: 9 * P * 4 + P * 8, lambda P: P),
}
PASSES = [
    ("fetch", ["FETCH_SIZE"]),
    ("write", ["WRITE_SIZE"]),
    ("sq", ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU",
            "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VMEM_RD", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]),
]


def child(name, P, reps):
    import torch
    from federated_amd import _lib
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    f32 = lambda: torch.randn(P, device="cuda", generator=g)
    f64 = lambda: torch.randn(P, device="cuda", generator=g, dtype=torch.float64)
    if name == "mix_seq_n8":
        local, out, nb = f32(), torch.empty(P, device="cuda"), [f32() for _ in range(8)]
        fn = lambda: eng.mix_seq(out, local, nb, [1.0 / 9] * 8)
    elif name == "mix_seq_div_n8":
        local, out, nb = f32(), torch.empty(P, device="cuda"), [f32() for _ in range(8)]
        fn = lambda: eng.mix_seq_div(out, local, nb, [1.0] * 8, [8.0] * 8)
    elif name == "compress_epilogue_mode2":
        y, ref, kept = f32(), f32(), eng.counter()
        fn = lambda: eng.compress(y, ref, 2, kept)
    elif name == "fold_f64_div_n4":
        l64, o64, nb64 = f64(), torch.empty(P, device="cuda", dtype=torch.float64), [f64() for _ in range(4)]
        fn = lambda: eng.fold_f64(o64, l64, nb64, [1.0] * 4, _lib.RULE_SEQUENTIAL_DIV, [4.0] * 4)
    elif name == "mewma_tf1_f64_n2":
        W64, s64, g64 = f64(), [f64() for _ in range(2)], [f64() for _ in range(2)]
        fn = lambda: eng.mewma_tf1_f64(W64, s64, g64, 0.99, 0.1, 0.1, P // 2, False, True)
    elif name == "mix_tf1_n8":
        local, out, nb = f32(), torch.empty(P, device="cuda"), [f32() for _ in range(8)]
        fn = lambda: eng.mix_tf1(out, local, nb, [1.0 / 9] * 8)
    elif name == "mix_tf1_wide_n8":
        local, nb = f32(), [f32() for _ in range(8)]
        o64 = torch.empty(P, device="cuda", dtype=torch.float64)
        tb, al64 = _lib.ptr_table([x.data_ptr() for x in nb]), _lib.double_array([1.0 / 9] * 8)
        fn = lambda: _lib.call("cfa_mix_tf1_wide_f32", o64.data_ptr(), local.data_ptr(), tb, al64, 8, P, 0, 0, 0,
                               None, eng.stream_handle())
    else:
        raise SystemExit(f"unknown kernel row {name}")
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"row": name, "avg_launch_ms": a.elapsed_time(b) / reps}), flush=True)


def per_dispatch(path):
    """{kernel name: {counter: [value per dispatch]}} from a counter_collection.csv."""
    acc = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "")
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            d = acc.setdefault(k, {}).setdefault(row["Counter_Name"], {})
            d[key] = d.get(key, 0.0) + float(row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in acc.items()}


def ours(kernels):
    """The library kernel of a child run: the non-torch kernel with the most dispatches."""
    cand = [(len(next(iter(cs.values()))), k) for k, cs in kernels.items() if "at::" not in k and cs]
    if not cand:
        return None
    return max(cand)[1]


def run_pass(name, counters, P, reps, workdir, timeout):
    prof = shutil.which("rocprofv3")
    d = os.path.join(workdir, f"{name}_{counters[0]}")
    cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", *counters, "-d", d, "-o", "pmc",
           "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--child", name,
           "--params", str(P), "--reps", str(reps)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    timing = None
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            timing = json.loads(line)
    if r.returncode != 0 or not files:
        return None, timing, f"rc {r.returncode}: {r.stderr[-400:]}"
    kernels = per_dispatch(files[0])
    k = ours(kernels)
    if k is None:
        return None, timing, "no library kernel in the pass"
    return (k, {c: statistics.median(v) for c, v in kernels[k].items()},
            {c: len(v) for c, v in kernels[k].items()}), timing, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", default=None)
    ap.add_argument("--params", type=int, default=P_DEFAULT)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--kernels", default=",".join(ROWS))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc_rows"))
    ap.add_argument("--pass-timeout", type=int, default=120)
    a = ap.parse_args()
    if a.child:
        child(a.child, a.params, a.reps)
        return
    os.makedirs(a.out, exist_ok=True)
    P = a.params
    results = []
    with tempfile.TemporaryDirectory(prefix="cfa_pmcrows_") as work:
        for name in a.kernels.split(","):
            entry, alg, elems = ROWS[name]
            row = {"row": name, "entry": entry, "params": P, "algorithmic_bytes": alg(P)}
            vals, errors, ms = {}, {}, []
            for pname, counters in PASSES:
                res, timing, err = run_pass(name, counters, P, a.reps, work, a.pass_timeout)
                if timing:
                    ms.append(timing["avg_launch_ms"])
                if err:
                    errors[pname] = err
                    if "rc 137" in err or "rc 124" in err:  # a killed pass: stop profiling
                        row["errors"] = errors
                        results.append(row)
                        print(json.dumps(row), flush=True)
                        raise SystemExit(2)
                    continue
                kname, med, count = res
                row["kernel"] = kname
                vals.update(med)
                row.setdefault("dispatches", {}).update(count)
            if ms:  # event time of the child's launches while counters were collected: not a rate
                row["avg_launch_ms_under_pmc"] = round(statistics.median(ms), 4)
            if "GRBM_GUI_ACTIVE" in vals:  # summed over the 8 XCDs: busy cycles of one launch
                row["gui_active_cycles_per_xcd"] = round(vals["GRBM_GUI_ACTIVE"] / 8.0, 1)
            row["counters"] = vals
            if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
                rd, wr = 2.0 * vals["FETCH_SIZE"] * 1024.0, vals["WRITE_SIZE"] * 1024.0
                row["hbm_read_bytes"], row["hbm_write_bytes"] = rd, wr
                row["traffic_over_algorithmic"] = round((rd + wr) / alg(P), 5)
            wc = vals.get("SQ_WAVE_CYCLES")
            if wc:
                row["valu_issue_frac_of_wave_time"] = round(vals.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, 4)
                row["wait_frac_of_wave_time"] = round(vals.get("SQ_WAIT_ANY", 0.0) / wc, 4)
                row["any_issue_frac_of_wave_time"] = round(vals.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 4)
            if "SQ_INSTS_VALU" in vals:
                row["valu_insts_per_64_elems"] = round(vals["SQ_INSTS_VALU"] / (elems(P) / 64.0), 3)
            if errors:
                row["errors"] = errors
            results.append(row)
            print(json.dumps(row), flush=True)
    with open(os.path.join(a.out, "pmc_rows.jsonl"), "w") as fh:
        for r in results:
            fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
