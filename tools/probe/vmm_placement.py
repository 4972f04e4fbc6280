#!/usr/bin/env python3
"""Does the way a stack is mapped decide its placement level (DESIGN §3 "Placement variance")?
The bench's population layout (an [L, 25M] fp32 input stack read by ring-window mixes of K = 8,
an [L, 25M] output stack written) allocated C times per method:

- torch: the caching allocator (what the bench uses);
- vmm_whole / vmm_1G / vmm_2M: one reserved VA range backed by physical handles of the whole
  size, of 1 GiB or of 2 MiB (hipMemCreate + hipMemMap, libcfa_exp's cfa_experimental_vmm_alloc).

Whole rounds per (method, candidate), interleaved over passes; pass 0 (first touch) is reported
apart. One JSON line per candidate, then a summary per method."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P, L = 25_000_000, int(os.environ.get("PROBE_L", "64"))
C, PASSES = int(os.environ.get("PROBE_C", "3")), int(os.environ.get("PROBE_PASSES", "4"))
METHODS = os.environ.get("PROBE_METHODS", "torch,vmm_whole,vmm_1G,vmm_2M").split(",")
eng = get_engine(0)
lib = _lib.load_experiments()
lib.cfa_experimental_vmm_alloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_int]
lib.cfa_experimental_vmm_free.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
lib.cfa_experimental_vmm_granularity.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t),
                                                 ctypes.POINTER(ctypes.c_size_t)]
CHUNK = {"vmm_whole": 0, "vmm_1G": 1 << 30, "vmm_64M": 64 << 20, "vmm_2M": 2 << 20}
alphas = [1.0 / 9] * 8
gmin, grec = ctypes.c_size_t(), ctypes.c_size_t()
assert lib.cfa_experimental_vmm_granularity(0, ctypes.byref(gmin), ctypes.byref(grec)) == 0, lib.cfa_exp_last_error()
print(json.dumps({"granularity_min": gmin.value, "granularity_recommended": grec.value}), flush=True)


class Vmm:
    def __init__(self, n, chunk):
        self.ptr, self.bytes, self.chunk = ctypes.c_void_p(), n * 4, chunk
        rc = lib.cfa_experimental_vmm_alloc(ctypes.byref(self.ptr), self.bytes, chunk, 0)
        if rc:
            raise RuntimeError(lib.cfa_exp_last_error())
        self.__cuda_array_interface__ = {"shape": (L, P), "typestr": "<f4", "data": (self.ptr.value, False),
                                         "version": 3, "strides": None}

    def free(self):
        lib.cfa_experimental_vmm_free(self.ptr, self.bytes, self.chunk, 0)


def stack(method, keep):
    if method.startswith("torch"):
        return torch.empty((L, P), device="cuda")
    v = Vmm(L * P, CHUNK[method])
    keep.append(v)
    return torch.as_tensor(v, device="cuda")


cands, keep = {}, []
for m in METHODS:
    for c in range(C):
        try:
            i, o = stack(m, keep), stack(m, keep)
        except RuntimeError as e:
            print(json.dumps({"method": m, "candidate": c, "error": str(e)}), flush=True)
            break
        i.normal_()
        cands[(m, c)] = [eng.prepare_mix_seq(o[d], i[d], [i[(d + k) % L] for k in (-4, -3, -2, -1, 1, 2, 3, 4)],
                                             alphas) for d in range(L)]
times = {k: [] for k in cands}
for _ in range(PASSES):
    for k, fns in cands.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for fn in fns:
            fn(None)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) * 1e3 / L)
by = {}
for (m, c), ts in times.items():
    med = statistics.median(ts[1:])
    by.setdefault(m, []).append(med)
    print(json.dumps({"experiment": "tools/probe/vmm_placement.py", "method": m, "candidate": c,
                      "first_touch_us": round(ts[0], 2), "us_per_mix": [round(t, 2) for t in ts[1:]],
                      "median_us": round(med, 2)}), flush=True)
for m, v in by.items():
    print(json.dumps({"experiment": "tools/probe/vmm_placement.py", "summary": m, "medians_us": [round(x, 2) for x in v],
                      "spread_us": round(max(v) - min(v), 2)}), flush=True)
for v in keep:
    v.free()
