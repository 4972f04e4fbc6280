#!/usr/bin/env python3
"""Does a side thread's hipMemcpyAsync enqueue wait while the main thread copies synchronously?

The host lane's receive side is enqueued by a pump thread (federated_amd/hostlane.py,
csrc/cfa_lane.cpp) while the round's own thread may sit in the transport. With the gloo
rehearsal's host-staged transport that thread runs synchronous device<->pageable copies
(`tensor.cpu()`); if the HIP runtime holds a lock through such a copy, the pump's enqueues wait
for it and the lane's H2D stream starves. This probe times a side thread's 4 MiB pinned H2D
enqueues (the call alone, not the copy) while the main thread is (a) idle, (b) doing pageable
`.cpu()` copies of 6.25 MB (the rehearsal's gloo pieces), (c) doing the same copies through a
pinned buffer on its own stream + that stream's synchronize. One JSON line: per phase the
median / p90 / max enqueue time (µs) and the main thread's copies per second.

Usage (GPU box): python tools/probe/enqueue_contention.py"""
import ctypes
import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from federated_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.Stream(dev)
    h = torch.empty(1 << 20, dtype=torch.float32, pin_memory=True)  # 4 MiB
    d = torch.empty(1 << 20, dtype=torch.float32, device=dev)
    src = torch.randn(6_250_000 // 4, device=dev)
    pinned = torch.empty(src.numel(), dtype=torch.float32, pin_memory=True)
    torch.cuda.synchronize()
    out = {}

    def run_phase(name, work):
        stop = threading.Event()
        lat = []

        def pump():
            torch.cuda.set_device(dev)
            while not stop.is_set():
                t0 = time.perf_counter()
                _lib.check("memcpy", lib.cfa_memcpy_async(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(h.data_ptr()),
                                                          h.numel() * 4, ctypes.c_void_p(side.cuda_stream)))
                lat.append((time.perf_counter() - t0) * 1e6)
                side.synchronize()
                time.sleep(0.0005)
        th = threading.Thread(target=pump)
        th.start()
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            work()
            n += 1
        stop.set()
        th.join()
        lat.sort()
        out[name] = {"enqueue_us_median": round(statistics.median(lat), 1),
                     "enqueue_us_p90": round(lat[int(0.9 * (len(lat) - 1))], 1),
                     "enqueue_us_max": round(lat[-1], 1), "samples": len(lat),
                     "main_copies_per_s": round(n / (time.perf_counter() - t0), 1)}

    run_phase("idle", lambda: time.sleep(0.001))
    run_phase("pageable_cpu_copies", lambda: src.cpu())

    def pinned_copy():
        with torch.cuda.stream(main_s):
            pinned.copy_(src, non_blocking=True)
        main_s.synchronize()
    run_phase("pinned_stream_copies", pinned_copy)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
