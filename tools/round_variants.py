#!/usr/bin/env python3
"""How to issue one consensus round of L device mixes (8 x 25M fp32 each): a single stream,
round-robin over S streams, a hipGraph replay of the single-stream round, and (for reference)
the one-launch population kernel. Interleaved rounds in one process; prints JSON lines with
the round time and the algorithmic GB/s."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.population import RingPopulationShard, RingShardPlan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--devices", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    eng = get_engine(0)
    plan = RingShardPlan(0, 1, a.devices, 4)
    shard = RingPopulationShard(plan, a.params, torch.device("cuda", 0), None, eng)
    shard.models.normal_()
    L = plan.L
    srcs = [shard.sources(i) for i in range(L)]
    main_s = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in range(4)]

    def one_stream():
        for i in range(L):
            eng.mix_seq(shard.mixed[i], shard.models[i], srcs[i], shard.alphas, main_s)

    def multi(S):
        def f():
            for s in streams[:S]:
                s.wait_stream(main_s)
            for i in range(L):
                eng.mix_seq(shard.mixed[i], shard.models[i], srcs[i], shard.alphas, streams[i % S])
            for s in streams[:S]:
                main_s.wait_stream(s)
        return f

    # population kernel tables (reference only: it can reuse neighbour reads through L2/MALL)
    ptrs = torch.tensor([shard.models[i].data_ptr() for i in range(L)], dtype=torch.int64, device="cuda")
    outs = torch.tensor([shard.mixed[i].data_ptr() for i in range(L)], dtype=torch.int64, device="cuda")
    ptr, idx, coef = [0], [], []
    for i in range(L):
        idx += [i] + plan.neighbours(i)
        coef += [1.0] + shard.alphas
        ptr.append(len(idx))
    cp = torch.tensor(ptr, dtype=torch.int32, device="cuda")
    ci = torch.tensor(idx, dtype=torch.int32, device="cuda")
    cc = torch.tensor(coef, dtype=torch.float32, device="cuda")

    def population():
        eng.population(outs, ptrs, cp, ci, cc, L, 0, a.params, main_s)

    # hipGraph of the single-stream round
    g = torch.cuda.CUDAGraph()
    one_stream()
    torch.cuda.synchronize()
    cap = torch.cuda.Stream()
    cap.wait_stream(main_s)
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            for i in range(L):
                eng.mix_seq(shard.mixed[i], shard.models[i], srcs[i], shard.alphas, cap)
    torch.cuda.synchronize()

    variants = {"one_stream": one_stream, "streams2": multi(2), "streams4": multi(4),
                "graph": lambda: g.replay(), "population_kernel": population}
    ref = None
    times = {k: [] for k in variants}
    for r in range(a.rounds):
        for k, f in variants.items():
            f()
            torch.cuda.synchronize()
            if r == 0:
                if ref is None:
                    ref = shard.mixed.clone()
                else:
                    assert torch.equal(shard.mixed, ref), k
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            f()
            e1.record(main_s)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    B = shard.bytes_per_round
    for k, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"variant": k, "round_ms_median": round(med, 3), "round_ms_min": round(min(ts), 3),
                          "per_mix_us": round(med * 1e3 / L, 2), "GBps": round(B / (med * 1e-3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
