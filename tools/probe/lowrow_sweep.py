#!/usr/bin/env python3
"""Round 4: the three lowest roofline rows (fp64 divisor fold, fp64 MEWMA, standalone compression)
against variants built on the headline mix's skeleton (tools/experiments/cfa_experiments.hip,
"the lowest roofline rows"): full tiles without per-vector guards, U 16-byte vectors per stream
per lane, a chosen store policy and workgroups per CU. Every variant's output is first checked
bit for bit against the production entry point on the same fresh inputs, then all variants and the
production kernel are timed on the same 25M-element HBM buffers, interleaved over PASSES passes
of REPS back-to-back launches (HIP events; median per variant).

Each row also gives the bytes each CU has in flight at its launch shape (workgroups per CU x 256
lanes x 16 B x vectors per stream x streams loaded per tile), to set against the guide's
~32 KiB-per-CU streaming figure (MI355X_MICROARCH.md).

"ceilings": the same skeleton with the lightest arithmetic (cfa_experimental_rw: R streams read,
W written, in place or not) at each kernel's read:write mix -- a float4 copy (1:1), the headline
mix (9:1), the fp64 fold (5:1), the standalone compression (2:1 in place) and the fp64 MEWMA (5:3,
three in place) -- over every instantiated shape; the best is what the chip streams at that mix.

Usage: python tools/probe/lowrow_sweep.py [--params 25000000] [--reps 20] [--passes 3]
           [--only fold,mewma,compress,ceilings]
Prints one JSON line per (kernel, variant)."""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

PEAK = 8000.0
LANES = 256


def timed(fn, reps, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def sweep(name, bytes_, variants, reps, passes, streams_loaded):
    """variants: [(label, fn, (bpc, u) or None for production)]; prints rows, returns them."""
    t = {lab: [] for lab, _, _ in variants}
    for _ in range(passes):
        for lab, fn, _ in variants:
            t[lab].append(timed(fn, reps))
    rows = []
    for lab, _, shape in variants:
        ms = statistics.median(t[lab])
        gbs = bytes_ / (ms * 1e-3) / 1e9
        r = {"kernel": name, "variant": lab, "avg_launch_ms": round(ms, 5), "GBps": round(gbs, 1),
             "frac": round(gbs / PEAK, 4), "passes_ms": [round(x, 5) for x in t[lab]]}
        if shape:
            bpc, u = shape
            r["inflight_KiB_per_CU"] = round(bpc * LANES * 16 * u * streams_loaded / 1024, 1)
        rows.append(r)
        print(json.dumps(r), flush=True)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--only", default="fold,mewma,compress,ceilings")
    a = ap.parse_args()
    from federated_amd import _lib
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    exp = _lib.load_experiments()
    P, R = a.params - a.params % 4, a.reps
    sh = eng.stream_handle()
    g = torch.Generator(device="cuda").manual_seed(7)
    f64 = lambda: torch.randn(P, device="cuda", generator=g, dtype=torch.float64)
    f32 = lambda: torch.randn(P, device="cuda", generator=g)
    vp = ctypes.c_void_p

    def call(fn, *args):
        rc = getattr(exp, fn)(*args)
        if rc != 0:
            raise RuntimeError(f"{fn}: {exp.cfa_exp_last_error().decode()}")

    only = set(a.only.split(","))
    if "fold" in only:
        n = 4
        loc, out, ref = f64(), torch.empty(P, device="cuda", dtype=torch.float64), torch.empty(P, device="cuda", dtype=torch.float64)
        nb = [f64() for _ in range(n)]
        al, dv = [1.0] * n, [4.0] * n
        tb = _lib.ptr_table([x.data_ptr() for x in nb])
        ad, dd = _lib.double_array(al), _lib.double_array(dv)
        prod = lambda: eng.fold_f64(out, loc, nb, al, _lib.RULE_SEQUENTIAL_DIV, dv)
        prod()
        torch.cuda.synchronize()
        ref.copy_(out)
        variants = [("production (2 WG/CU, U=2, sc1 buffer store, full tiles)", prod, (2, 2))]
        for bpc, u, sp in [(1, 2, 2), (2, 2, 2), (1, 2, 1), (2, 2, 1), (2, 1, 1), (4, 1, 1), (2, 2, 3),
                           (1, 4, 2), (2, 1, 2), (4, 1, 2), (1, 1, 3), (1, 4, 3), (2, 4, 3), (4, 4, 3), (1, 2, 3),
                           (4, 2, 3)]:
            fn = (lambda bpc=bpc, u=u, sp=sp: call("cfa_experimental_fold64_div", vp(out.data_ptr()), vp(loc.data_ptr()),
                                                   tb, ad, dd, ctypes.c_size_t(P), u, sp, bpc, vp(sh)))
            out.zero_()
            fn()
            torch.cuda.synchronize()
            if not torch.equal(out, ref):
                raise SystemExit(f"fold64 variant bpc={bpc} u={u} sp={sp} differs from production")
            variants.append((f"bpc={bpc} u={u} sp={sp}", fn, (bpc, u)))
        sweep("cfa_fold_f64 (divisor rule, n=4)", (n + 2) * P * 8, variants, R, a.passes, n + 1)
        del loc, out, ref, nb
        torch.cuda.empty_cache()
    if "mewma" in only:
        W0, s0 = f64(), [f64() for _ in range(2)]
        gg = [f64() for _ in range(2)]
        W, s = W0.clone(), [x.clone() for x in s0]
        rho, lr1, lr2, split = 0.99, 0.1, 0.1, P // 2
        prod = lambda: eng.mewma_tf1_f64(W, s, gg, rho, lr1, lr2, split, False, True)

        def reset():
            W.copy_(W0)
            for x, y in zip(s, s0):
                x.copy_(y)
        reset()
        prod()
        torch.cuda.synchronize()
        Wr, sr = W.clone(), [x.clone() for x in s]
        st = _lib.ptr_table([x.data_ptr() for x in s])
        gt = _lib.ptr_table([x.data_ptr() for x in gg])
        variants = [("production (1 WG/CU, U=1, nt loads/stores)", prod, (1, 1))]
        for bpc, u, sp, ntl in [(1, 2, 1, 1), (1, 2, 2, 1), (2, 1, 1, 1), (2, 2, 1, 1), (1, 1, 2, 1),
                                (2, 1, 2, 1), (1, 2, 0, 0), (2, 1, 0, 0), (1, 1, 3, 1), (4, 1, 1, 1),
                                (2, 1, 3, 1), (2, 2, 3, 1), (1, 2, 3, 1), (1, 1, 3, 0), (2, 1, 3, 0),
                                (4, 4, 3, 1), (2, 4, 3, 1), (1, 4, 3, 1), (4, 2, 3, 1), (1, 4, 1, 1), (2, 4, 1, 1),
                                (1, 4, 2, 1),
                                # sp + 10: stream-major load / store order (mewma64_sm_kernel)
                                (1, 1, 11, 1), (1, 2, 11, 1), (1, 4, 11, 1), (1, 4, 13, 1), (2, 4, 13, 1),
                                (4, 4, 13, 1), (2, 2, 13, 1), (1, 4, 12, 1), (2, 4, 11, 1),
                                # sp + 20: software-pipelined (mewma64_pipe_kernel, round 4)
                                (1, 1, 21, 1), (2, 1, 21, 1), (1, 2, 21, 1), (1, 1, 23, 1), (2, 1, 23, 1),
                                (1, 2, 23, 1), (2, 2, 23, 1), (1, 1, 22, 1), (2, 1, 22, 1), (4, 1, 21, 1),
                                (1, 4, 23, 1), (1, 1, 20, 0), (2, 1, 20, 0)]:
            fn = (lambda bpc=bpc, u=u, sp=sp, ntl=ntl: call(
                "cfa_experimental_mewma64", vp(W.data_ptr()), st, gt, ctypes.c_double(rho), ctypes.c_double(lr1),
                ctypes.c_double(lr2), ctypes.c_size_t(split), 1, ctypes.c_size_t(P), u, sp, ntl, bpc, vp(sh)))
            reset()
            fn()
            torch.cuda.synchronize()
            if not (torch.equal(W, Wr) and all(torch.equal(x, y) for x, y in zip(s, sr))):
                raise SystemExit(f"mewma64 variant bpc={bpc} u={u} sp={sp} ntl={ntl} differs from production")
            variants.append((f"bpc={bpc} u={u} sp={sp} ntl={ntl}", fn, (bpc, u)))
        sweep("cfa_mewma_tf1_f64 (n=2)", (3 * 2 + 2) * P * 8, variants, R, a.passes, 5)
        del W0, s0, gg, W, s, Wr, sr
        torch.cuda.empty_cache()
    if "compress" in only:
        y0, loc = f32(), f32()
        y = y0.clone()
        kept = eng.counter()
        prod = lambda: eng.compress(y, loc, 2, kept)
        prod()
        torch.cuda.synchronize()
        yr, kr = y.clone(), int(kept.item())
        variants = [("production (2 WG/CU, U=4, default policy, compile-time mode form)", prod, (2, 4))]
        for bpc, u, sp, ntl in [(2, 4, 0, 0), (4, 4, 0, 0), (2, 8, 0, 0), (4, 2, 0, 0), (2, 4, 1, 1),
                                (2, 4, 2, 1), (2, 4, 3, 0), (1, 8, 0, 0), (2, 4, 1, 0), (4, 4, 2, 1)]:
            fn = (lambda bpc=bpc, u=u, sp=sp, ntl=ntl: call(
                "cfa_experimental_compress_full", vp(y.data_ptr()), vp(loc.data_ptr()), ctypes.c_size_t(P), 2,
                vp(kept.data_ptr()), u, sp, ntl, bpc, vp(sh)))
            y.copy_(y0)
            kept.zero_()
            fn()
            torch.cuda.synchronize()
            if not (torch.equal(y, yr) and int(kept.item()) == kr):
                raise SystemExit(f"compress variant bpc={bpc} u={u} sp={sp} ntl={ntl} differs from production")
            variants.append((f"bpc={bpc} u={u} sp={sp} ntl={ntl}", fn, (bpc, u)))
        sweep("cfa_compress_epilogue_f32 (mode 2)", 3 * P * 4, variants, R, a.passes, 2)
        del y0, loc, y, yr
        torch.cuda.empty_cache()
    if "ceilings" in only:
        # (label, reads, writes, writes in place over the first reads)
        mixes = [("copy 1:1", 1, 1, False), ("headline mix 9:1", 9, 1, False), ("fp64 fold 5:1 (n=4)", 5, 1, False),
                 ("compression 2:1, in place", 2, 1, True), ("fp64 MEWMA 5:3, three in place (n=2)", 5, 3, True)]
        shapes = [(u, sp, ntl) for u, sp, ntl in [(1, 1, 1), (2, 1, 1), (4, 1, 1), (2, 3, 1), (4, 3, 1), (2, 2, 1),
                                                   (4, 0, 0), (2, 0, 0), (4, 3, 0), (1, 3, 1)]]
        for label, r, w, inplace in mixes:
            srcs = [f32() for _ in range(r)]
            dsts = srcs[:w] if inplace else [torch.empty(P, device="cuda") for _ in range(w)]
            st_ = _lib.ptr_table([x.data_ptr() for x in srcs])
            dt_ = _lib.ptr_table([x.data_ptr() for x in dsts])
            variants = []
            for bpc in (1, 2, 4):
                for u, sp, ntl in shapes:
                    fn = (lambda bpc=bpc, u=u, sp=sp, ntl=ntl: call(
                        "cfa_experimental_rw", st_, dt_, r, w, ctypes.c_size_t(P), u, sp, ntl, bpc, vp(sh)))
                    variants.append((f"bpc={bpc} u={u} sp={sp} ntl={ntl}", fn, (bpc, u)))
            rows = sweep(f"ceiling: {label}", (r + w) * P * 4, variants, R, a.passes, r)
            best = max(rows, key=lambda x: x["frac"])
            print(json.dumps({"ceiling": label, "reads": r, "writes": w, "in_place": inplace, "best_variant": best["variant"],
                              "best_frac": best["frac"], "best_GBps": best["GBps"]}), flush=True)
            del srcs, dsts
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
