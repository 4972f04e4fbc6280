#!/usr/bin/env python3
"""How a tiny zero-copy launch's completion is awaited: hipStreamSynchronize (blocking) against
spinning on hipStreamQuery, for the C1-shaped fp32 plan and a device-resident launch."""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.consensus import _runtime as R  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

hip = None
for path in _lib.loaded_hip_runtimes():
    hip = ctypes.CDLL(path)
hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
hip.hipStreamQuery.restype = ctypes.c_int
for fn in ("hipEventRecord", "hipEventSynchronize", "hipEventQuery"):
    getattr(hip, fn).restype = ctypes.c_int
hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
hip.hipEventQuery.argtypes = [ctypes.c_void_p]
hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
hip.hipEventCreateWithFlags.restype = ctypes.c_int
ev_default, ev_nt = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipEventCreateWithFlags(ctypes.byref(ev_default), 0) == 0
assert hip.hipEventCreateWithFlags(ctypes.byref(ev_nt), 2) == 0  # hipEventDisableTiming


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
st = mx._stream()
plan = mx._zc_plan("f32", R._layout_of(local), 2, np.float32)
sh = plan.stream_handle(st)
co = plan.coeffs(al)
L = plan.lib


def zc_launch():
    L.cfa_mix_seq_f32(plan.ob, plan.hb, plan.table, co, 2, plan.P, sh)


eng = get_engine(0)
d = [torch.randn(plan.P, device="cuda") for _ in range(3)]
dout = torch.empty(plan.P, device="cuda")
dev_launch = eng.prepare_mix_seq(dout, d[0], d[1:], al)


def dev_go():
    dev_launch(st)


def spin():
    while hip.hipStreamQuery(sh) != 0:
        pass


def block():
    L.cfa_stream_synchronize(sh)


res = {"experiment": "tools/probe/sync_latency.py"}
res["launch_only_us"] = med(zc_launch, 200)
block()
res["zc_launch_block_us"] = med(lambda: (zc_launch(), block()))
res["zc_launch_spin_us"] = med(lambda: (zc_launch(), spin()))
res["dev_launch_block_us"] = med(lambda: (dev_go(), block()))
res["dev_launch_spin_us"] = med(lambda: (dev_go(), spin()))
res["query_idle_us"] = med(lambda: hip.hipStreamQuery(sh))


def ev_sync(ev):
    hip.hipEventRecord(ev, sh)
    hip.hipEventSynchronize(ev)


def ev_spin(ev):
    hip.hipEventRecord(ev, sh)
    while hip.hipEventQuery(ev) != 0:
        pass


res["zc_launch_event_sync_us"] = med(lambda: (zc_launch(), ev_sync(ev_default)))
res["zc_launch_event_nt_sync_us"] = med(lambda: (zc_launch(), ev_sync(ev_nt)))
res["zc_launch_event_spin_us"] = med(lambda: (zc_launch(), ev_spin(ev_nt)))
res["zc_launch_block_again_us"] = med(lambda: (zc_launch(), block()))
print(json.dumps(res))
