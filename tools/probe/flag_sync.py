#!/usr/bin/env python3
"""Completion of a small zero-copy drop-in call (C1 fp32 plan: P = 16 680, 2 neighbours): the
production launch + hipStreamSynchronize against waiting on a pinned host word that the GPU sets
after the mix (tools/experiments/cfa_experiments.hip: hipStreamWriteValue32, a one-lane flag
kernel, or the mix kernel itself with a last-workgroup signal). Each variant's output is checked
against the production result. GPU box: python tools/probe/flag_sync.py"""
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

X = _lib.load_experiments()
X.cfa_experimental_signal.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_int]
X.cfa_experimental_wait_flag.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_longlong]
X.cfa_experimental_mix2_flag.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint,
                                         ctypes.c_void_p]
X.cfa_experimental_signal_inc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
for fn in ("cfa_experimental_signal", "cfa_experimental_wait_flag", "cfa_experimental_mix2_flag",
           "cfa_experimental_signal_inc"):
    getattr(X, fn).restype = ctypes.c_int


def med(fn, n=1000):
    for _ in range(50):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2), round(min(ts) * 1e6, 2)


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
eng = get_engine(0)
flag_t = torch.zeros(16, dtype=torch.int32, pin_memory=True)
flag_host = flag_t.data_ptr()
flag_dev = eng.host_device_ptr(flag_t)
counter = torch.zeros(16, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
seq = [0]
# pack once: rows hold the local model and the two neighbours
for m, arrs in enumerate([local] + nbrs):
    for k, a in enumerate(arrs):
        np.copyto(plan.views[m][k], a.ravel())


def base():
    L.cfa_mix_seq_f32(plan.ob, plan.hb, plan.table, co, 2, plan.P, sh)
    L.cfa_stream_synchronize(sh)


def signalled(method):
    def go():
        seq[0] += 1
        L.cfa_mix_seq_f32(plan.ob, plan.hb, plan.table, co, 2, plan.P, sh)
        X.cfa_experimental_signal(sh, flag_dev, seq[0], method)
        assert X.cfa_experimental_wait_flag(flag_host, seq[0], 1 << 34) == 0
    return go


def fused():
    seq[0] += 1
    X.cfa_experimental_mix2_flag(plan.ob, plan.hb, plan.table, co, plan.P, counter.data_ptr(), flag_dev, seq[0], sh)
    assert X.cfa_experimental_wait_flag(flag_host, seq[0], 1 << 34) == 0


# graph variant: the mix and a counter-bumping signal kernel captured once, replayed per call
gflag_t = torch.zeros(16, dtype=torch.int32, pin_memory=True)
gflag_host, gflag_dev = gflag_t.data_ptr(), eng.host_device_ptr(gflag_t)
gcounter = torch.zeros(16, dtype=torch.int32, device="cuda")
gs = torch.cuda.Stream()
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph, stream=gs):
    L.cfa_mix_seq_f32(plan.ob, plan.hb, plan.table, co, 2, plan.P, gs.cuda_stream)
    X.cfa_experimental_signal_inc(gs.cuda_stream, gcounter.data_ptr(), gflag_dev)
torch.cuda.synchronize()
gseq = [int(gflag_t[0])]


def graphed():
    gseq[0] += 1
    graph.replay()
    assert X.cfa_experimental_wait_flag(gflag_host, gseq[0], 1 << 34) == 0


base()
ref = plan.out_np.copy()
for name, fn in [("write_value32", signalled(0)), ("flag_kernel", signalled(1)), ("fused_last_block", fused),
                 ("graph_mix_and_signal", graphed)]:
    plan.out_np[:] = 0
    L.cfa_stream_synchronize(sh)
    fn()
    same = bool(np.array_equal(plan.out_np, ref))
    L.cfa_stream_synchronize(sh)
    print(json.dumps({"check": name, "equal_after_flag": same}), flush=True)

rows = {}
for rep in range(3):
    for name, fn in [("hipStreamSynchronize", base), ("write_value32", signalled(0)),
                     ("flag_kernel", signalled(1)), ("fused_last_block", fused),
                     ("graph_mix_and_signal", graphed)]:
        rows.setdefault(name, []).append(med(fn))
        L.cfa_stream_synchronize(sh)
for name, v in rows.items():
    print(json.dumps({"experiment": "tools/probe/flag_sync.py", "variant": name, "P": plan.P, "n": 2,
                      "median_us_per_call": [x[0] for x in v], "min_us": [x[1] for x in v]}), flush=True)
