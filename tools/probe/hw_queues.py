#!/usr/bin/env python3
"""Do two HIP streams of one process share a hardware queue (and so block each other)?

HIP maps streams onto at most GPU_MAX_HW_QUEUES hardware queues per process (4 by default);
streams beyond that share a queue, and a queue runs its packets in order. A kernel that waits
(the host lane's cfa_stream_wait_word, or an RCCL kernel waiting for its peer) then also holds
back every other stream on its queue. This probe creates ``--streams`` torch streams, parks a
wait kernel on stream 0 (it waits for a pinned host word the host raises after ``--hold-ms``), and
for every other stream launches a tiny kernel and times from its enqueue to its completion: a
stream that shares stream 0's queue completes only after the word is raised. One JSON line:
per stream, completed before the release (independent queue) or not (shared).

Usage (GPU box): [GPU_MAX_HW_QUEUES=n] python tools/probe/hw_queues.py [--streams 8]"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--hold-ms", type=float, default=300.0)
    a = ap.parse_args()
    import torch
    from federated_amd import _lib
    lib = _lib.load()
    word = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    status = torch.zeros(16, dtype=torch.int32, pin_memory=True)

    def dev(t):
        p = ctypes.c_void_p()
        _lib.check("ptr", lib.cfa_host_device_pointer(ctypes.c_void_p(t.data_ptr()), ctypes.byref(p)))
        return p.value
    wd, sd = dev(word), dev(status)
    streams = [torch.cuda.Stream() for _ in range(a.streams)]
    x = torch.zeros(1024, device="cuda")
    torch.cuda.synchronize()
    res = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "streams": a.streams, "shares_with_0": []}
    for i in range(1, a.streams):
        word.zero_()
        _lib.check("wait", lib.cfa_stream_wait_word(ctypes.c_void_p(wd), 1, int(10e6), ctypes.c_void_p(sd),
                                                    ctypes.c_void_p(streams[0].cuda_stream)))
        time.sleep(0.01)  # the wait kernel is running
        ev = torch.cuda.Event()
        with torch.cuda.stream(streams[i]):
            x.add_(1.0)
            ev.record(streams[i])
        t0 = time.perf_counter()
        done_early = False
        while time.perf_counter() - t0 < a.hold_ms * 1e-3:
            if ev.query():
                done_early = True
                break
            time.sleep(0.0005)
        word[0] = 1  # release stream 0
        torch.cuda.synchronize()
        res["shares_with_0"].append({"stream": i, "independent": done_early})
    res["shared_count"] = sum(1 for r in res["shares_with_0"] if not r["independent"])
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
