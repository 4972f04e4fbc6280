#!/usr/bin/env python3
"""Where an N = 2 round with the host lane spends its time, host side and GPU side.

Two processes on the visible GPU (the bench's one-GPU rehearsal), gloo for the link pieces, the
full bench shape (128 devices x 25M, K = 8) and the bench's route (planned on fixed rates: gloo
at ``--link-gbps`` and the lane at ``--lane-gbps``, which gives the `measured+lane` plan of the
rehearsals). After warm-up, ``--rounds`` timed rounds, each traced:

* host: when the round's thread enters and leaves the lane's ``run``, every transport group, the
  interior mixes, every gate wait (a boundary set waiting for its lane rows) and ``finish``
  (ms from the round's start);
* GPU: HIP events on the compute stream at the round's start and end, on the comm stream after
  each group, and the lane's own per-group events on its in stream (ms from the round's start).

One JSON line per rank with the medians over the rounds.

Usage (GPU box): python tools/probe/lane_round_trace.py [--rounds 5] [--placement 1]"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def child(rank, world, port, a, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd import hostlane
        from federated_amd.dist import TorchTransport
        from federated_amd.engine import get_engine
        from federated_amd.halo import LANE_IN, LANE_OUT
        from federated_amd.linkprobe import agree_gloo
        from federated_amd.population import make_ring_shard
        from federated_amd.streams import role_stream
        tok = [hostlane.new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        rates = {(x, y): a.link_gbps for x in range(world) for y in range(world) if x != y}
        rates.update({(x, LANE_OUT): a.lane_gbps for x in range(world)})
        rates.update({(LANE_IN, x): a.lane_gbps for x in range(world)})
        eng = get_engine(0)
        tr = TorchTransport()
        shard, info = make_ring_shard(rank, world, 128, 4, 4, a.params, torch.device("cuda", 0), tr, eng,
                                      link_rates=rates, lane_token=tok[0], lane_agree=agree_gloo,
                                      placement_candidates=a.placement)
        for i in range(shard.plan.L):
            shard.models[i].normal_(generator=torch.Generator(device="cuda").manual_seed(7 + shard.plan.first + i))
        cs, ms = torch.cuda.current_stream(), role_stream("comm")
        lane = shard.lane
        trace = []
        t_round = [0.0]

        def wrap(obj, name, label, **fixed):
            fn = getattr(obj, name)

            def w(*args, **kw):
                kw.update(fixed)
                t0 = time.perf_counter()
                try:
                    return fn(*args, **kw)
                finally:
                    trace.append((label, (t0 - t_round[0]) * 1e3, (time.perf_counter() - t_round[0]) * 1e3))
            setattr(obj, name, w)
        wrap(lane, "run", "lane.run", timing=True)  # timed events, so their landing can be read
        wrap(lane, "finish", "lane.finish")
        wrap(tr, "exchange", "gloo group")
        gate_wait = hostlane.LaneGate.wait

        def gw(self, stream=None):
            t0 = time.perf_counter()
            try:
                return gate_wait(self, stream)
            finally:
                trace.append((f"gate {self.group}", (t0 - t_round[0]) * 1e3, (time.perf_counter() - t_round[0]) * 1e3))
        hostlane.LaneGate.wait = gw
        mix_set = shard._mix_set
        interior = set(shard.interior_order())

        def ms_wrap(devices, stream, timer=None, between=None):
            t0 = time.perf_counter()
            mix_set(devices, stream, timer, between)
            trace.append(("interior mixes" if set(devices) <= interior and len(devices) > 4 else "boundary mixes",
                          (t0 - t_round[0]) * 1e3, (time.perf_counter() - t_round[0]) * 1e3))
        shard._mix_set = ms_wrap
        for _ in range(a.warmup):
            shard.round(cs, ms)
        torch.cuda.synchronize()
        dist.barrier()
        rounds = []
        for _ in range(a.rounds):
            trace.clear()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t_round[0] = time.perf_counter()
            e0.record(cs)
            shard.round(cs, ms)
            e1.record(cs)
            host_ms = (time.perf_counter() - t_round[0]) * 1e3
            torch.cuda.synchronize()
            rnd = lane._last_round
            gpu = {"round_end": e0.elapsed_time(e1)}
            for g, e in (rnd.events or {}).items():
                gpu[f"lane group {g} landed"] = e0.elapsed_time(e)
            rounds.append({"host_ms": host_ms, "trace": list(trace), "gpu": gpu})
        # medians per trace label occurrence
        out = {"rank": rank, "plan": info["route_choice"]["chosen"], "lane_MB": info["route"]["lane_elems"] * 4 / 1e6,
               "round_gpu_ms": round(statistics.median(r["gpu"]["round_end"] for r in rounds), 3),
               "round_host_ms": round(statistics.median(r["host_ms"] for r in rounds), 3)}
        keys = [(lab, i) for i, (lab, _, _) in enumerate(rounds[0]["trace"])]
        out["host"] = [{"what": lab, "start_ms": round(statistics.median(r["trace"][i][1] for r in rounds), 3),
                        "end_ms": round(statistics.median(r["trace"][i][2] for r in rounds), 3)}
                       for lab, i in keys if all(len(r["trace"]) > i for r in rounds)]
        out["gpu"] = {k: round(statistics.median(r["gpu"][k] for r in rounds), 3) for k in rounds[0]["gpu"]}
        q.put(out)
        shard.close()
    except Exception as exc:
        q.put({"rank": rank, "error": f"{type(exc).__name__}: {exc}"})
    finally:
        dist.destroy_process_group()


def main():
    import multiprocessing as mp
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--placement", type=int, default=1)
    ap.add_argument("--link-gbps", type=float, default=1.24)
    ap.add_argument("--lane-gbps", type=float, default=21.0)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 37100 + os.getpid() % 997
    procs = [ctx.Process(target=child, args=(r, 2, port, a, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for r in sorted(res, key=lambda x: x["rank"]):
        print(json.dumps(r), flush=True)
    return 0 if all("error" not in r for r in res) else 1


if __name__ == "__main__":
    sys.exit(main())
