#!/usr/bin/env python3
"""Do the rank's streams hold each other back at the box's hardware-queue count?

HIP maps a process's streams onto at most GPU_MAX_HW_QUEUES hardware queues (4 on this pool);
streams beyond that share a queue, and a queue runs its packets in order. Round 5 measured this
with a wait kernel parked on one stream (`profiles/r05_hw_queues.jsonl`: at 4 queues one of 7
streams stalled behind it) and raised the queue count; round 6 removed every wait from the GPU
queues (the host lane waits on the host, federated_amd/hostlane.py) and runs at the pool's
setting. What is left to check is whether ordinary work on one of the rank's streams delays a
tiny kernel on another: for each pair (A, B) of the rank's stream budget (compute = torch's
current stream, and federated_amd.streams' comm, lane_out, lane_in), each used once first, a long
piece of work goes on A (a 1 GiB H2D copy from pinned memory for the lane streams, ~20 ms; 60
element-wise kernels over 1 GiB, ~25 ms, for compute / comm), then a tiny kernel on B; B is
independent when its kernel completes before A's work does. One JSON line.

Usage (GPU box): [GPU_MAX_HW_QUEUES=n] python tools/probe/hw_queues.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from federated_amd.streams import role_stream
    dev = torch.device("cuda", torch.cuda.current_device())
    roles = {"compute": torch.cuda.current_stream(dev)}
    for r in ("comm", "lane_out", "lane_in"):
        roles[r] = role_stream(r, dev)
    host = torch.empty(1 << 28, dtype=torch.float32, pin_memory=True)  # 1 GiB
    big = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    x = torch.zeros(1024, device=dev)
    for s in roles.values():  # every stream used once first (its queue bound, its first launch paid)
        with torch.cuda.stream(s):
            x.add_(1.0)
            big.copy_(host, non_blocking=True)
    torch.cuda.synchronize()

    def long_work(s, role):
        with torch.cuda.stream(s):
            if role.startswith("lane"):
                big.copy_(host, non_blocking=True)
            else:
                for _ in range(60):  # ~25 ms of HBM-bound kernels
                    big.mul_(1.0001)

    res = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "pairs": []}
    for a, sa in roles.items():
        for b, sb in roles.items():
            if a == b:
                continue
            done_a = torch.cuda.Event()
            long_work(sa, a)
            done_a.record(sa)
            ev = torch.cuda.Event()
            with torch.cuda.stream(sb):
                x.add_(1.0)
                ev.record(sb)
            t0 = time.perf_counter()
            first = None
            while time.perf_counter() - t0 < 2.0:
                qb, qa = ev.query(), done_a.query()
                if qb or qa:
                    first = "b" if qb and not qa else ("a" if qa and not qb else "both")
                    break
                time.sleep(0.0002)
            torch.cuda.synchronize()
            res["pairs"].append({"long_on": a, "tiny_on": b, "tiny_first": first == "b"})
    res["held_back"] = [f"{p['tiny_on']} behind {p['long_on']}" for p in res["pairs"] if not p["tiny_first"]]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
