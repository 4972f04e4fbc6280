#!/usr/bin/env python3
"""What differs between an allocation at the fast placement level and one at the slow level?

Child mode (`--child`, run under rocprofv3 --pmc): allocates PAIRS (input rows, output) pairs
carved from 16 GiB allocations (as placement.calibrated_stacks does), then for each pair in turn
runs WARM + REPS production K = 8 x 25M mixes (HIP events around the REPS), and prints one JSON
line with every pair's time per mix and the dispatch order (pair p owns mix dispatches
[p * (WARM + REPS), (p + 1) * (WARM + REPS))).

Parent mode (default): runs the child under rocprofv3 once per counter pass (pass 1: UTCL1
translation requests / hits / misses and the TCP->TCC read latency; pass 2: the TCC's DRAM
credit stalls for reads and writes, UTCL2 busy and GUI-active cycles), attributes each
dispatch's counters to its pair by order, and prints per pair: the mix time in that pass and the
median of each counter. If the slow pairs show more translation misses, the level is address
translation; if more DRAM credit stalls at equal translation behaviour, it is the memory side.

Usage (GPU box): python tools/probe/level_counters.py [--pairs 4] [--out gpurun_out/level_counters]"""
import argparse
import glob
import json
import os
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
KERNEL = "mix_vec_kernel<8, 0, 2, 2>"
PASSES = [
    ("tlb", ["TCP_UTCL1_TRANSLATION_MISS_sum", "TCP_UTCL1_TRANSLATION_HIT_sum", "TCP_UTCL1_REQUEST_sum",
             "TCP_TCC_READ_REQ_LATENCY_sum"]),
    ("dram", ["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "GRBM_UTCL2_BUSY",
              "GRBM_GUI_ACTIVE"]),
]


def child(pairs, warm, reps):
    import torch
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    P, K = 25_000_000, 8
    hold, fns = [], []
    for _ in range(pairs):
        big_in = torch.empty(16 << 28, device="cuda")
        big_out = torch.empty(16 << 28, device="cuda")
        hold += [big_in, big_out]
        ins = big_in[:(K + 1) * P].view(K + 1, P).normal_()
        fns.append(eng.prepare_mix_seq(big_out[:P], ins[0], [ins[j] for j in range(1, K + 1)], [1.0 / (K + 1)] * K))
    torch.cuda.synchronize()
    times = []
    for fn in fns:
        for _ in range(warm):
            fn(None)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn(None)
        b.record()
        b.synchronize()
        times.append(round(a.elapsed_time(b) * 1e3 / reps, 2))
    print(json.dumps({"pair_mix_us": times, "per_pair_dispatches": warm + reps}), flush=True)


def parent(a):
    os.makedirs(a.out, exist_ok=True)
    out = {"passes": {}}
    for name, counters in PASSES:
        d = os.path.join(a.out, name)
        cmd = ["rocprofv3", "--pmc"] + counters + ["-d", d, "-o", name, "--output-format", "csv", "--",
                                                     sys.executable, os.path.abspath(__file__), "--child",
                                                     "--pairs", str(a.pairs)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.pass_timeout)
        info = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files or not info:
            out["passes"][name] = {"error": f"rc {r.returncode}", "stderr": r.stderr[-800:]}
            print(json.dumps(out), flush=True)
            return 1
        import csv
        rows = [x for x in csv.DictReader(open(files[0])) if KERNEL in x["Kernel_Name"]]
        per = info[0]["per_pair_dispatches"]
        by_dispatch = {}
        for x in rows:
            by_dispatch.setdefault(int(x["Dispatch_Id"]), {})[x["Counter_Name"]] = float(x["Counter_Value"])
        ids = sorted(by_dispatch)
        res = []
        for p in range(a.pairs):
            mine = ids[p * per:(p + 1) * per]
            res.append({"pair": p, "mix_us_in_pass": info[0]["pair_mix_us"][p],
                        **{c: statistics.median(by_dispatch[i].get(c, float("nan")) for i in mine) for c in counters}})
        out["passes"][name] = res
    print(json.dumps(out), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "level_counters"))
    ap.add_argument("--pass-timeout", type=int, default=120)
    a = ap.parse_args()
    if a.child:
        child(a.pairs, a.warm, a.reps)
        return 0
    return parent(a)


if __name__ == "__main__":
    sys.exit(main())
