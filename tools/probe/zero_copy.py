#!/usr/bin/env python3
"""Host-resident K = 8 x 25M mix with the mix kernel reading its buckets straight from pinned
host memory and writing the result straight back (no staging copies: PCIe reads and the write
run in the two link directions at once), against the copy-based serial / pipelined forms of
staging.measure_e2e. Device pointers of the pinned buffers come from hipHostGetDevicePointer;
if the runtime does not map them, the probe stops before any launch."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.staging import measure_e2e  # noqa: E402

P, K, REPS = 25_000_000, 8, 5
eng = get_engine(0)
hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
hip.hipHostGetDevicePointer.restype = ctypes.c_int


def devptr(t):
    p = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), 0)
    if rc != 0 or not p.value:
        print(json.dumps({"probe": "zero_copy", "error": f"hipHostGetDevicePointer rc={rc}"}), flush=True)
        sys.exit(0)
    return p.value


host_in = [torch.empty(P, dtype=torch.float32, pin_memory=True).normal_() for _ in range(K + 1)]
host_out = torch.empty(P, dtype=torch.float32, pin_memory=True)
dp_in = [devptr(h) for h in host_in]
dp_out = devptr(host_out)
alphas = [1.0 / (K + 1)] * K
s = torch.cuda.current_stream()

ref = torch.empty(P, device="cuda")
d_in = [h.cuda() for h in host_in]
eng.mix_seq(ref, d_in[0], d_in[1:], alphas)
del d_in


def zc(launch):
    lc = _lib.Launch(*launch)
    _lib.call("cfa_mix_seq_ex_f32", dp_out, dp_in[0], _lib.ptr_table(dp_in[1:]), _lib.float_array(alphas), K, P,
              ctypes.addressof(lc), int(s.cuda_stream))


rows = [{"probe": "zero_copy", "variant": "copies", **measure_e2e(eng, P, K)}]
for launch in [(2, 4, 1), (8, 4, 1), (16, 4, 1), (8, 1, 1), (16, 1, 0)]:
    host_out.zero_()
    zc(launch)
    torch.cuda.synchronize()
    same = bool(torch.equal(host_out.cuda(), ref))
    t0 = time.perf_counter()
    for _ in range(REPS):
        zc(launch)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / REPS
    rows.append({"probe": "zero_copy", "variant": "kernel_on_pinned_host", "launch": launch, "ms": round(dt * 1e3, 3),
                 "algorithmic_GBps": round((K + 2) * P * 4 / dt / 1e9, 2), "equals_device_result": same})
for r in rows:
    print(json.dumps(r), flush=True)
