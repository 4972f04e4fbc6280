#!/usr/bin/env python3
"""HostMixer.mix at the TF2 drop-in sizes: the single-shot zero-copy path (pack everything, one
PCIe kernel) against the Python chunk pipeline (pack chunk c + 1 while the kernel reads chunk c)
and the native one (cfa_host_mix_f32: the same overlap in one libcfa call, host copy threads)
at several chunk sizes and thread counts. Medians of whole calls.
Usage: python tools/probe/pipeline_threshold.py [--native-only]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from federated_amd.consensus import _runtime as R  # noqa: E402

CASES = {
    "syn_1MB": ([(65_536,)], 3),
    "syn_2MB": ([(131_072,)], 3),
    "syn_4MB": ([(262_144,)], 3),
    "c1": ([(512, 32), (32,), (32, 8), (8,)], 2),
    "c4": ([(3, 3, 3, 32), (32,), (3, 3, 32, 32), (32,), (8192, 128), (128,), (128, 100), (100,)], 4),
    "radar": ([(8, 8, 1, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (7168, 512), (512,),
               (512, 6), (6,)], 2),
    "ps_c4": ([(3, 3, 3, 32), (32,), (3, 3, 32, 32), (32,), (8192, 128), (128,), (128, 100), (100,)], 8),
    "radar_k8": ([(8, 8, 1, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (7168, 512), (512,),
                  (512, 6), (6,)], 8),
}


def med(fn, reps):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    mx = R.mixer()
    for case, (shapes, n) in CASES.items():
        rng = np.random.default_rng(0)
        local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
        nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(n)]
        al = [1.0 / (n + 1)] * n
        P = sum(int(np.prod(s)) for s in shapes)
        reps = 200 if P < 100_000 else 40
        row = {"experiment": "tools/probe/pipeline_threshold.py", "case": case, "P": P, "n": n,
               "staging_MB": round((n + 1) * P * 4 / 1e6, 1)}
        R.NATIVE_PIPELINE = False
        R.PIPELINE_MIN_BYTES = 1 << 62
        ref = mx.mix(local, nbrs, al)[0]
        row["single_shot_us"] = med(lambda: mx.mix(local, nbrs, al), reps)
        if "--native-only" not in sys.argv:
            R.PIPELINE_MIN_BYTES = 0
            for chunk_mb in (16,):
                R.PIPELINE_CHUNK_BYTES = chunk_mb << 20
                out = mx.mix(local, nbrs, al)[0]
                assert all(np.array_equal(x, y) for x, y in zip(out, ref))
                row[f"pipeline_{chunk_mb}MB_us"] = med(lambda: mx.mix(local, nbrs, al), reps)
        R.PIPELINE_MIN_BYTES, R.PIPELINE_CHUNK_BYTES = 64 << 20, 128 << 20
        lay = R._layout_of(local)
        for chunk in (64 << 10, 128 << 10, 256 << 10, 512 << 10):
            for th in (4, 8):
                fn = lambda: mx._mix_native(lay, local, nbrs, al, None, chunk_elems=chunk, threads=th)
                assert all(np.array_equal(x, y) for x, y in zip(fn(), ref))
                row[f"native_{chunk >> 10}K_t{th}_us"] = med(fn, reps)
        R.NATIVE_PIPELINE = True
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
