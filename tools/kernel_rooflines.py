#!/usr/bin/env python3
"""Roofline of every libcfa streaming kernel at a large bucket (HBM-bound regime).

Each entry point runs back to back on HBM-resident buckets (HIP events around `--reps`
launches after warm-up). Its algorithmic bytes per launch are the DESIGN.md §3 formula, so
achieved GB/s = bytes / average launch time, and frac = that over the 8 TB/s HBM3E spec peak.
Prints one JSON line per kernel. Usage: python tools/kernel_rooflines.py [--params 25000000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = 8000.0


BPC_VARIANTS = []  # --bpc-variants: workgroups per CU compared on the same buffers (CFA_TUNE_DYNAMIC)


def _timed_once(fn, reps, warm):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps  # ms


def timed(fn, reps, warm=3):
    """ms per launch; with --bpc-variants a dict {workgroups per CU: ms}, the variants
    interleaved over three passes on the same buffers (median per variant)."""
    if not BPC_VARIANTS:
        return _timed_once(fn, reps, warm)
    import statistics
    t = {v: [] for v in BPC_VARIANTS}
    for _ in range(3):
        for v in BPC_VARIANTS:  # "B" = workgroups per CU, "B:V" = also float4 per lane
            b, _, vec = str(v).partition(":")
            os.environ["CFA_BLOCKS_PER_CU"] = b
            if vec:
                os.environ["CFA_VEC_PER_LANE"] = vec
            else:
                os.environ.pop("CFA_VEC_PER_LANE", None)
            t[v].append(_timed_once(fn, reps, warm))
    os.environ.pop("CFA_BLOCKS_PER_CU", None)
    os.environ.pop("CFA_VEC_PER_LANE", None)
    return {v: statistics.median(x) for v, x in t.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ballast-gib", type=int, default=0,
                    help="hold this much device memory (touched) for the whole run before any bucket is "
                         "allocated, so the buckets do not land on a process's first-allocation memory "
                         "(the slow placement level, DESIGN §3)")
    ap.add_argument("--bpc-variants", default="",
                    help="comma list of workgroups per CU (optionally :float4 per lane) to compare on the "
                         "same buffers, e.g. 2,1 or 1:2,1:4 "
                         "(sets CFA_TUNE_DYNAMIC before the library loads)")
    a = ap.parse_args()
    if a.bpc_variants:
        os.environ["CFA_TUNE_DYNAMIC"] = "1"
        BPC_VARIANTS.extend(a.bpc_variants.split(","))
    ballast = None
    if a.ballast_gib:
        ballast = torch.empty(a.ballast_gib << 28, dtype=torch.float32, device="cuda")
        ballast.zero_()
    from federated_amd import _lib
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    P, R = a.params, a.reps
    g = torch.Generator(device="cuda").manual_seed(1)
    f32 = lambda: torch.randn(P, device="cuda", generator=g)
    f64 = lambda: torch.randn(P, device="cuda", generator=g, dtype=torch.float64)
    rows = []

    def rec(name, entry, bytes_, ms, note=""):
        if isinstance(ms, dict):
            for v, m in ms.items():
                rec(name, entry, bytes_, m, (note + "; " if note else "") + f"blocks_per_cu={v}")
            return
        gbs = bytes_ / (ms * 1e-3) / 1e9
        r = {"kernel_entry": entry, "case": name, "params": P, "avg_launch_ms": round(ms, 4),
             "algorithmic_bytes": bytes_, "GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4)}
        if note:
            r["note"] = note
        rows.append(r)
        print(json.dumps(r), flush=True)

    n = 8
    local, out = f32(), torch.empty(P, device="cuda")
    nb = [f32() for _ in range(n)]
    al = [1.0 / (n + 1)] * n
    rec("sequential mix, n=8", "cfa_mix_seq_f32", (n + 2) * P * 4, timed(lambda: eng.mix_seq(out, local, nb, al), R))
    rec("FedAvg divisor fold, n=8", "cfa_mix_seq_div_f32", (n + 2) * P * 4,
        timed(lambda: eng.mix_seq_div(out, local, nb, [1.0] * n, [float(n)] * n), R))
    rec("linear closed form, n=8", "cfa_mix_f32", (n + 2) * P * 4,
        timed(lambda: eng.mix_linear(out, local, nb, [0.1] * (n + 1)), R))
    rec("TF1 rule, fp32 buckets, n=8", "cfa_mix_tf1_f32", (n + 2) * P * 4,
        timed(lambda: eng.mix_tf1(out, local, nb, al), R))
    o64w = torch.empty(P, device="cuda", dtype=torch.float64)
    tb = _lib.ptr_table([x.data_ptr() for x in nb])
    al64 = _lib.double_array(al)
    rec("TF1 rule, fp32 buckets in, unrounded fp64 out, n=8", "cfa_mix_tf1_wide_f32", (n + 1) * P * 4 + P * 8,
        timed(lambda: _lib.call("cfa_mix_tf1_wide_f32", o64w.data_ptr(), local.data_ptr(), tb, al64, n, P, 0, 0, 0,
                                None, eng.stream_handle()), R))
    del o64w
    kept = eng.counter()
    rec("mix + fused compression (mode 2) on the whole bucket, n=3", "cfa_mix_seq_compress_f32", 5 * P * 4,
        timed(lambda: eng.mix_seq_compress(out, local, nb[:3], al[:3], 2, 0, P, kept), R))
    rec("standalone compression epilogue (mode 2)", "cfa_compress_epilogue_f32", 3 * P * 4,
        timed(lambda: eng.compress(out, local, 2, kept), R))
    W, s2, g2 = f32(), [f32() for _ in range(2)], [f32() for _ in range(2)]
    rec("MEWMA update, n=2", "cfa_mewma_update_f32", (3 * 2 + 2) * P * 4,
        timed(lambda: eng.mewma(W, s2, g2, 0.99, 0.1, 0.1, P // 2, False, True), R))
    del nb, s2, g2
    torch.cuda.empty_cache()
    n64 = 4
    l64, o64 = f64(), torch.empty(P, device="cuda", dtype=torch.float64)
    nb64 = [f64() for _ in range(n64)]
    rec("TF1 rule, fp64 buckets, n=4", "cfa_mix_tf1_f64", (n64 + 2) * P * 8,
        timed(lambda: eng.mix_tf1_f64(o64, l64, nb64, [0.25] * n64, False), R))
    rec("fp64 fold (FedAvg divisor), n=4", "cfa_fold_f64", (n64 + 2) * P * 8,
        timed(lambda: eng.fold_f64(o64, l64, nb64, [1.0] * n64, _lib.RULE_SEQUENTIAL_DIV, [4.0] * n64), R))
    W64, s64, g64 = f64(), [f64() for _ in range(2)], [f64() for _ in range(2)]
    rec("MEWMA on fp64 buckets, n=2", "cfa_mewma_tf1_f64", (3 * 2 + 2) * P * 8,
        timed(lambda: eng.mewma_tf1_f64(W64, s64, g64, 0.99, 0.1, 0.1, P // 2, False, True), R))
    del nb64, s64, g64, W64, l64, o64
    torch.cuda.empty_cache()
    # population: 16 devices, 4 random neighbours each, one launch
    D, K = 16, 4
    models = torch.randn(D, P, device="cuda", generator=g)
    mixed = torch.empty_like(models)
    rng = np.random.default_rng(0)
    lists = [[int(j) for j in rng.choice([k for k in range(D) if k != d], K, replace=False)] for d in range(D)]
    ptr = np.zeros(D + 1, np.int32)
    idx, coef = [], []
    for d, l in enumerate(lists):
        idx += [d] + l
        coef += [0.0] + [0.2] * K
        ptr[d + 1] = len(idx)
    t = lambda v, dt: torch.tensor(v, dtype=dt, device="cuda")
    src = t([models[d].data_ptr() for d in range(D)], torch.int64)
    dst = t([mixed[d].data_ptr() for d in range(D)], torch.int64)
    tabs = (t(ptr, torch.int32), t(idx, torch.int32), t(coef, torch.float32))
    rec("population round, 16 devices x 4 random neighbours", "cfa_mix_population_f32", D * (K + 2) * P * 4,
        timed(lambda: eng.population(dst, src, *tabs, D, _lib.RULE_SEQUENTIAL, P), R // 2),
        "rows shared between devices may hit the Infinity Cache: algorithmic bytes can exceed HBM traffic")
    # fused CFA-GE step: 16 devices, their 4 neighbours, MEWMA states and gradients per entry
    S = torch.randn(len(idx), P, device="cuda", generator=g)
    G = torch.randn(len(idx), P, device="cuda", generator=g)
    states = t([0 if k in ptr[:-1] else S[k].data_ptr() for k in range(len(idx))], torch.int64)
    grads = t([0 if k in ptr[:-1] else G[k].data_ptr() for k in range(len(idx))], torch.int64)
    srcge = t([models[d].data_ptr() for d in range(D)] * 2, torch.int64)
    rec("CFA-GE population step, 16 devices x 4 neighbours (mix + MEWMA fused)", "cfa_ge_population_step_f32",
        D * (4 * K + 2) * P * 4,
        timed(lambda: eng.ge_population_step(dst, srcge, states, grads, *tabs, D, 0.99, 0.1, 0.1, P // 2, True, P),
              R // 2),
        "neighbour rows shared between devices may hit the Infinity Cache")
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                           "kernel_rooflines.jsonl"), "w") as fh:
        for r in rows:
            fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
