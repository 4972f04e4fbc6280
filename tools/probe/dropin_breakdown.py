#!/usr/bin/env python3
"""Breakdown of one zero-copy drop-in call: pack, launch + sync, unpack, for the fp32 plan
(HostMixer.mix) and the fp64 plan (HostMixer.mix_tf1). Medians over 500 calls (50 above 1M
parameters). Usage: python tools/probe/dropin_breakdown.py [c1|c4|radar]  (c4: VGG-1 with 4
neighbours, radar: the TF2 radar CNN with 2)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.consensus import _runtime as R  # noqa: E402


def med(fn, n=500):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2)


CASES = {
    "c1": ([(512, 32), (32,), (32, 8), (8,)], 2),
    "c4": ([(3, 3, 3, 32), (32,), (3, 3, 32, 32), (32,), (8192, 128), (128,), (128, 100), (100,)], 4),
    "radar": ([(8, 8, 1, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (7168, 512), (512,),
               (512, 6), (6,)], 2),
}
case = sys.argv[1] if len(sys.argv) > 1 else "c1"
shapes, N = CASES[case]
rng = np.random.default_rng(0)
local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(N)]
al = [1.0 / (N + 1)] * N
P = sum(int(np.prod(s)) for s in shapes)
if P > 1_000_000:
    med.__defaults__ = (50,)
mx = R.mixer()
mx.mix(local, nbrs, al)
mx.mix_tf1(local, nbrs, al)
st = mx._stream()
out = {}
for kind, dt in (("f32", np.float32), ("f64", np.float64)):
    plan = mx._zc_plan(kind, R._layout_of(local), N, dt)
    sh = plan.stream_handle(st)
    co = plan.coeffs(al, kind == "f64")
    if kind == "f32":
        launch = lambda: plan.lib.cfa_mix_seq_f32(plan.ob, plan.hb, plan.table, co, N, plan.P, sh)
    else:
        tb = plan.run_table(0)
        launch = lambda: plan.lib.cfa_mix_tf1_f64(plan.ob, plan.hb, tb, co, N, 1, plan.P, 0, 0, 0, None, sh)
    sync = lambda: plan.lib.cfa_stream_synchronize(sh)
    out[kind] = {
        "pack_us": med(lambda: plan.pack(local, nbrs)),
        "launch_only_us": med(lambda: (launch(), sync())[0]) ,
        "sync_idle_us": med(sync),
        "unpack_us": med(plan.unpack),
        "layout_key_us": med(lambda: R._layout_of(local)),
        "full_call_us": med(lambda: mx.mix(local, nbrs, al) if kind == "f32" else mx.mix_tf1(local, nbrs, al)),
    }
print(json.dumps({"experiment": "tools/probe/dropin_breakdown.py", "case": case, "P": P, "n": N, **out}))
