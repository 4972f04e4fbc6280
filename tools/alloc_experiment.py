#!/usr/bin/env python3
"""Is the per-mix level (158 / 163 / 167 us, profiles/r01_placement.jsonl) a property of how the
buckets are allocated? Sliding-window rounds (K = 8, P = 25M) over 16 buckets + 16 outputs,
allocated three times per method: torch caching allocator, hipExtMallocWithFlags default (0),
contiguous (4), uncached (3). Interleaved rounds in one process."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P, L, R, REPS = 25_000_000, 16, 5, int(os.environ.get("ALLOC_REPS", "3"))
eng = get_engine(0)
lib = _lib.load_experiments()
lib.cfa_experimental_malloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
lib.cfa_experimental_free.argtypes = [ctypes.c_void_p]
a = [1.0 / 9] * 8


class Raw:
    """A hipExtMalloc'd fp32 buffer exposed to torch through __cuda_array_interface__."""

    def __init__(self, n, flags):
        self.ptr = ctypes.c_void_p()
        rc = lib.cfa_experimental_malloc(ctypes.byref(self.ptr), n * 4, flags)
        if rc:
            raise RuntimeError(lib.cfa_exp_last_error())
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (self.ptr.value, False),
                                         "version": 3, "strides": None}


keep = []


def buckets(method):
    if method == "torch":
        return [torch.empty(P, device="cuda") for _ in range(2 * L)]
    flags = {"hip_default": 0, "hip_finegrained": 1, "hip_contiguous": 4, "hip_uncached": 3}[method]
    out = []
    for _ in range(2 * L):
        r = Raw(P, flags)
        keep.append(r)
        out.append(torch.as_tensor(r, device="cuda"))
    return out


sets = {}
for method in os.environ.get("ALLOC_METHODS", "torch,hip_default,hip_contiguous,hip_uncached").split(","):
    for k in range(REPS):
        try:
            b = buckets(method)
        except RuntimeError as e:
            print(json.dumps({"method": method, "error": str(e)}), flush=True)
            break
        for t in b[:L]:
            t.normal_()
        sets[(method, k)] = (b[:L], b[L:])


def run(m, o):
    for i in range(L):
        eng.mix_seq(o[i], m[i], [m[(i + d) % L] for d in (-4, -3, -2, -1, 1, 2, 3, 4)], a)


times = {k: [] for k in sets}
for _ in range(R):
    for key, (m, o) in sets.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(m, o)
        e1.record()
        torch.cuda.synchronize()
        times[key].append(e0.elapsed_time(e1) / L)
for (method, k), ts in times.items():
    med = statistics.median(ts)
    print(json.dumps({"method": method, "alloc": k, "us_per_mix": round(med * 1e3, 2),
                      "GBps": round(1e9 / (med * 1e-3) / 1e9, 1)}), flush=True)
