#!/usr/bin/env python3
"""Mixes under CU contention (the N > 1 compute term of DESIGN §5): 16 back-to-back 8-neighbour
mixes (P = 25M) on one stream while a bounded copy kernel holding `blocks` workgroups runs on
another stream (a stand-in for RCCL's copy kernels during a halo exchange). Static grid-stride
tiles (production) against dynamic tiles (one device counter, experiment kernel)."""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd import _lib  # noqa: E402
from federated_amd.engine import get_engine  # noqa: E402

P, K, M = 25_001_984, 8, 16
eng = get_engine(0)
exp = _lib.load_experiments()
exp.cfa_experimental_mix8_dyn.restype = ctypes.c_int
exp.cfa_experimental_mix8_dyn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                          ctypes.POINTER(ctypes.c_float), ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_void_p]
exp.cfa_experimental_hog.restype = ctypes.c_int
exp.cfa_experimental_hog.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p]
xs = [torch.randn(P, device="cuda") for _ in range(K + 1)]
outs = [torch.empty(P, device="cuda") for _ in range(2)]
al = [1.0 / (K + 1)] * K
prod = [eng.prepare_mix_seq(o, xs[0], xs[1:], al) for o in outs]
tab = _lib.ptr_table([x.data_ptr() for x in xs[1:]])
alc = _lib.float_array(al)
ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
A, B = torch.cuda.current_stream(), torch.cuda.Stream()
hn = 64 << 20  # floats: 256 MB
hsrc, hdst = torch.randn(hn, device="cuda"), torch.empty(hn, device="cuda")


def dyn(o, st):
    rc = exp.cfa_experimental_mix8_dyn(o.data_ptr(), xs[0].data_ptr(), tab, alc, P, ctr.data_ptr(), 2, st.cuda_stream)
    assert rc == 0


def run(kind, blocks, reps):
    B.wait_stream(A)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if blocks:
        assert exp.cfa_experimental_hog(hdst.data_ptr(), hsrc.data_ptr(), hn, blocks, reps, B.cuda_stream) == 0
    a.record(A)
    for m in range(M):
        if kind == "static":
            prod[m % 2](A)
        else:
            dyn(outs[m % 2], A)
    b.record(A)
    A.wait_stream(B)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / M * 1e3


def hog_time(blocks, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(B)
    exp.cfa_experimental_hog(hdst.data_ptr(), hsrc.data_ptr(), hn, blocks, reps, B.cuda_stream)
    b.record(B)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3


ref = torch.empty(P, device="cuda")
eng.mix_seq(ref, xs[0], xs[1:], al)
dyn(outs[0], A)
torch.cuda.synchronize()
assert torch.equal(outs[0], ref)
res = {"experiment": "tools/probe/contention.py", "mixes": M, "params": P}
cfg = {}
for blocks in (16, 32, 64):
    t1 = hog_time(blocks, 1)
    reps = max(1, int(1.3 * M * 165.0 / t1))  # outlasts the mixes
    cfg[blocks] = reps
    res[f"hog{blocks}_alone_us_per_rep"] = round(t1, 1)
rows = {}
for _ in range(5):
    for kind in ("static", "dynamic"):
        for blocks in (0, 16, 32, 64):
            rows.setdefault(f"{kind}_hog{blocks}", []).append(run(kind, blocks, cfg.get(blocks, 0)))
res["us_per_mix_median"] = {k: round(statistics.median(v), 2) for k, v in rows.items()}
print(json.dumps(res))
