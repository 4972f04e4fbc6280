#!/usr/bin/env python3
"""The N > 1 bench rank's round at its own bucket size: launch shape and launch mode.

At N > 1 the bench's headline partition (params) gives every rank a 1/N element slice of all 128
buckets, so a rank runs 128 mixes of P/N elements per round: 3.125M at N = 8, where a mix takes
about 20 us and the boundaries between launches weigh more than at 25M (152 us). This times one
ring round (K = 8, the bench population) on placement-calibrated stacks of the slice size for:

  - eager: the bench's own path (prepared launches, one foreign call per mix);
  - graph: the same round captured once as a hipGraph and replayed, for every launch shape of
    1/2/4 workgroups per CU x 1/2/4 float4 per lane (CFA_TUNE_DYNAMIC: the shape is read at capture).

Rounds are interleaved over passes; prints one JSON line per (P, variant) with the median time per
device mix and the algorithmic rate."""
import itertools
import json
import os
import statistics
import sys

os.environ["CFA_TUNE_DYNAMIC"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402
from federated_amd.placement import calibrated_stacks  # noqa: E402
from federated_amd.population import slice_bounds  # noqa: E402

PFULL, L = 25_000_000, 128
H = int(os.environ.get("SLICE_HALF", "4"))  # K = 2 H ring-window neighbours
PASSES = int(os.environ.get("SLICE_PASSES", "5"))
WORLDS = [int(x) for x in os.environ.get("SLICE_WORLDS", "8,4,2").split(",")]  # P = 25M / world
SIZES = [int(x) for x in os.environ.get("SLICE_SIZES", "").split(",") if x]  # explicit P values instead
BPC = [int(x) for x in os.environ.get("SLICE_BPC", "1,2,4").split(",")]
VEC = [int(x) for x in os.environ.get("SLICE_VEC", "1,2,4").split(",")]
CAND = int(os.environ.get("SLICE_CANDIDATES", "4"))
# ring: device d reads the ring window around row d (consecutive mixes share 2H of their 2H + 1
# input rows, which the Infinity Cache can serve at small P); scattered: device d reads rows
# (2H + 1) d .. (2H + 1) d + 2H (mod L), so consecutive mixes share no row and a row returns only ~L / (2H + 1)
# mixes later (no reuse from the 256 MB cache above ~1M elements)
PATTERN = os.environ.get("SLICE_PATTERN", "ring")
eng = get_engine(0)
alphas = [1.0 / (2 * H + 1)] * (2 * H)
offsets = list(range(-H, 0)) + list(range(1, H + 1))


def set_shape(bpc, vec):
    os.environ["CFA_BLOCKS_PER_CU"] = str(bpc)
    os.environ["CFA_VEC_PER_LANE"] = str(vec)


def clear_shape():
    os.environ.pop("CFA_BLOCKS_PER_CU", None)
    os.environ.pop("CFA_VEC_PER_LANE", None)


cases = [(0, P) for P in SIZES] if SIZES else [(w, slice_bounds(PFULL, w)[1]) for w in WORLDS]
for world, P in cases:
    m, o, rep = calibrated_stacks(L, P, "cuda", eng, H, H, candidates=CAND)
    m.normal_(generator=torch.Generator(device="cuda").manual_seed(3))
    if PATTERN == "ring":
        rows = [(d, [(d + k) % L for k in offsets]) for d in range(L)]
    else:
        st = 2 * H + 1
        rows = [((st * d) % L, [(st * d + 1 + j) % L for j in range(2 * H)]) for d in range(L)]
    fns = [eng.prepare_mix_seq(o[d], m[a], [m[j] for j in nb], alphas) for d, (a, nb) in enumerate(rows)]
    stream = torch.cuda.Stream()
    variants = {}

    def eager():
        for fn in fns:
            fn(stream)
    clear_shape()
    variants["eager_default"] = eager
    for bpc, vec in itertools.product(BPC, VEC):
        set_shape(bpc, vec)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            eager()  # warm the shape outside the capture
            stream.synchronize()
            g.capture_begin()
            eager()
            g.capture_end()
        variants[f"graph_bpc{bpc}_vec{vec}"] = g.replay
    clear_shape()
    times = {k: [] for k in variants}
    for _ in range(PASSES):
        for k, run in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record(stream)
                run()
                e1.record(stream)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / L)
    bytes_mix = (2 * H + 2) * P * 4
    for k in sorted(times, key=lambda k: statistics.median(times[k])):
        us = statistics.median(times[k])
        print(json.dumps({"experiment": "tools/probe/slice_shape.py", "world": world, "P": P, "devices": L, "neighbours": 2 * H, "pattern": PATTERN,
                          "variant": k, "us_per_device_mix": round(us, 3), "min_us": round(min(times[k]), 3),
                          "GBps": round(bytes_mix / (us * 1e-6) / 1e9, 1),
                          "placement_chosen_us": rep.get("chosen_us")}), flush=True)
    del m, o, fns, variants
    torch.cuda.empty_cache()
