#!/usr/bin/env python3
"""Breakdown of one zero-copy drop-in call at the C1 shapes: pack, launch + sync, unpack, for
the fp32 plan (HostMixer.mix) and the fp64 plan (HostMixer.mix_tf1). Medians over 500 calls."""
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


rng = np.random.default_rng(0)
shapes = [(512, 32), (32,), (32, 8), (8,)]
local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(2)]
al = [0.5, 0.5]
mx = R.mixer()
mx.mix(local, nbrs, al)
mx.mix_tf1(local, nbrs, al)
st = mx._stream()
out = {}
for kind, dt in (("f32", np.float32), ("f64", np.float64)):
    plan = mx._zc_plan(kind, R._layout_of(local), 2, dt)
    sh = plan.stream_handle(st)
    co = plan.coeffs(al, kind == "f64")
    if kind == "f32":
        launch = lambda: plan.lib.cfa_mix_seq_f32(plan.ob, plan.hb, plan.table, co, 2, plan.P, sh)
    else:
        tb = plan.run_table(0)
        launch = lambda: plan.lib.cfa_mix_tf1_f64(plan.ob, plan.hb, tb, co, 2, 1, plan.P, 0, 0, 0, None, sh)
    sync = lambda: plan.lib.cfa_stream_synchronize(sh)
    out[kind] = {
        "pack_us": med(lambda: plan.pack(local, nbrs)),
        "launch_only_us": med(lambda: (launch(), sync())[0]) ,
        "sync_idle_us": med(sync),
        "unpack_us": med(plan.unpack),
        "layout_key_us": med(lambda: R._layout_of(local)),
        "full_call_us": med(lambda: mx.mix(local, nbrs, al) if kind == "f32" else mx.mix_tf1(local, nbrs, al)),
    }
print(json.dumps({"experiment": "tools/probe/dropin_breakdown.py", "P": 16680, **out}))
