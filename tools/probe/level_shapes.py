#!/usr/bin/env python3
"""Does any launch shape of the headline mix recover the slow placement level?

The K = 8 x 25M sequential mix runs at one of a few rates (about 150 and 162 us) depending on the
allocation its stacks land on; since round 6 the bench's headline runs on plain
allocations, so a box whose allocation lands on the slow level reports it. This probe allocates
``--pairs`` plain (models, mixed) stack pairs of the bench's shape ([128, 25M] fp32 each, like
``RingPopulationShard``), times the ring-window mix of ``--rows`` spread devices on each with the
library's default shape and with explicit shapes (blocks per CU, float4 per lane, nontemporal),
passes interleaved across pairs and shapes, and prints one JSON line: per pair and shape the
median microseconds per mix. A shape that is fast on both levels would be a better default.

Usage (GPU box): python tools/probe/level_shapes.py [--pairs 4] [--rows 32] [--passes 3]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [None, (1, 1, 1), (1, 2, 1), (1, 4, 1), (2, 1, 1), (2, 2, 1), (4, 1, 1), (1, 2, 0), (2, 2, 0), (4, 2, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--rows", type=int, default=32)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--devices", type=int, default=128)
    ap.add_argument("--params", type=int, default=25_000_000)
    a = ap.parse_args()
    import torch
    from federated_amd.engine import get_engine
    eng = get_engine(0)
    L, P, h = a.devices, a.params, 4
    alphas = [1.0 / (2 * h + 1)] * (2 * h)
    offs = list(range(-h, 0)) + list(range(1, h + 1))
    gen = torch.Generator(device="cuda").manual_seed(20261015)
    pairs = []
    for _ in range(a.pairs):
        m = torch.empty((L, P), dtype=torch.float32, device="cuda")
        o = torch.empty((L, P), dtype=torch.float32, device="cuda")
        m.normal_(generator=gen)
        pairs.append((m, o))
    sel = sorted({(i * L) // a.rows for i in range(a.rows)})

    def timed(m, o, shape):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for d in sel:
            eng.mix_seq(o[d], m[d], [m[(d + k) % L] for k in offs], alphas, launch=shape)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / len(sel)

    for m, o in pairs:  # first touch of everything
        timed(m, o, None)
    t = {(p, s): [] for p in range(len(pairs)) for s in range(len(SHAPES))}
    for _ in range(a.passes):
        for s, shape in enumerate(SHAPES):
            for p, (m, o) in enumerate(pairs):
                t[(p, s)].append(timed(m, o, shape))
    out = {"rows": len(sel), "pairs": []}
    for p in range(len(pairs)):
        row = {"default_us": round(statistics.median(t[(p, 0)]), 2)}
        for s, shape in enumerate(SHAPES[1:], 1):
            row["bpc%d_vec%d_nt%d" % shape] = round(statistics.median(t[(p, s)]), 2)
        out["pairs"].append(row)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
