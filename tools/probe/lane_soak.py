#!/usr/bin/env python3
"""Soak of the host lane's cross-process protocol (federated_amd/hostlane.py) on the GPU.

Two processes on the visible GPU, each the sender of one direction and the receiver of the other,
exchange three lane messages per round (two groups, odd lengths and offsets, so the ramped chunks,
both parities and the ack back-pressure all turn over) for ``--rounds`` rounds. Every round each
sender fills its source rows with a value unique to (round, rank, message) on its compute stream,
then runs the lane on that stream; the receiver synchronises and checks every landed row against
the value its peer wrote (exact: a constant row). Random host delays of up to ``--jitter-ms``
between rounds shift the ranks against each other, so the receiver's waits and the sender's ack
waits both see real skew. Prints one JSON line: rounds, rows checked, mismatches, seconds.

Usage (GPU box): python tools/probe/lane_soak.py [--rounds 200] [--jitter-ms 3]"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

LENGTHS = [(0, 3_000_017), (0, 1_000_003), (1, 2_500_001)]  # (group, elements) per message


def value(r, rank, i):
    return float((r % 4096) * 16 + rank * 4 + i)


def child(rank, world, port, a, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.halo import ALIGN, Message
        from federated_amd.hostlane import HostLane, new_token
        from federated_amd.linkprobe import agree_gloo
        tok = [new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        offs, msgs = [], []
        off = 0
        for g, n in LENGTHS:
            offs.append(off)
            off += -(-n // ALIGN) * ALIGN + ALIGN
        src_buf = torch.zeros(off, device="cuda")
        dst_buf = torch.zeros(off, device="cuda")
        for s in range(world):
            for i, (g, n) in enumerate(LENGTHS):
                msgs.append(Message(g, s, 1 - s, "src", offs[i], "dst", offs[i], n, lane=True))
        bufs = {"src": src_buf, "dst": dst_buf}
        lane = HostLane.open(rank, [m for m in msgs if m.src == rank], [m for m in msgs if m.dst == rank],
                             lambda k: bufs[k], torch.device("cuda", 0), tok[0], agree_gloo,
                             chunk_elems=1 << 20, timeout_s=20.0)
        cs = torch.cuda.current_stream()
        rng = random.Random(1234 + rank)
        bad, rows = 0, 0
        t0 = time.perf_counter()
        for r in range(a.rounds):
            for i, (g, n) in enumerate(LENGTHS):
                src_buf[offs[i]:offs[i] + n].fill_(value(r, rank, i))
            lane.run(cs)
            lane.wait_streams(cs)
            cs.synchronize()
            lane.check()
            peer = 1 - rank
            for i, (g, n) in enumerate(LENGTHS):
                v = dst_buf[offs[i]:offs[i] + n]
                want = value(r, peer, i)
                rows += 1
                bad += int(not bool(((v == want).all()).item()))
            if a.jitter_ms > 0:
                time.sleep(rng.random() * a.jitter_ms * 1e-3)
        secs = time.perf_counter() - t0
        lane.close()
        q.put((rank, {"rounds": a.rounds, "rows_checked": rows, "mismatches": bad, "seconds": round(secs, 2)}))
    except Exception as exc:  # reported by the parent
        q.put((rank, {"error": f"{type(exc).__name__}: {exc}"}))
    finally:
        dist.destroy_process_group()


def main():
    import multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--jitter-ms", type=float, default=3.0)
    ap.add_argument("--wall-s", type=float, default=240.0)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 36500 + os.getpid() % 997
    procs = [ctx.Process(target=child, args=(r, 2, port, a, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=a.wall_s) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    print(json.dumps({"soak": res}), flush=True)
    ok = all("error" not in v and v["mismatches"] == 0 for v in res.values())
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
