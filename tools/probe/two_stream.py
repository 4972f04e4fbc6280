#!/usr/bin/env python3
"""Do back-to-back device mixes gain from alternating two streams (the tail of one launch
overlapping the head of the next)? 32 ring devices x 25M, K = 8, the production launch
(prepare_mix_seq), one stream vs two streams alternating, interleaved rounds."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from federated_amd.engine import get_engine  # noqa: E402

D, P, h = 32, 25_000_000, 4
eng = get_engine(0)
models = torch.randn(D, P, device="cuda")
mixed = torch.empty_like(models)
al = [1.0 / 9] * 8
launch = [eng.prepare_mix_seq(mixed[d], models[d], [models[(d + o) % D] for o in (-4, -3, -2, -1, 1, 2, 3, 4)], al)
          for d in range(D)]
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
ss = [torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()]


def one():
    for f in launch:
        f(s0)


def two():
    s1.wait_stream(s0)
    for d, f in enumerate(launch):
        f(s0 if d % 2 == 0 else s1)
    s0.wait_stream(s1)


def three():
    for s in ss[1:]:
        s.wait_stream(s0)
    streams = [s0] + ss[1:]
    for d, f in enumerate(launch):
        f(streams[d % 3])
    for s in ss[1:]:
        s0.wait_stream(s)


def timed(fn):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s0)
    fn()
    b.record(s0)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / D * 1e3  # us per device mix


res = {"one": [], "two": [], "three": []}
for fn in (one, two, three):
    fn()
torch.cuda.synchronize()
ref = mixed.clone()
for _ in range(6):
    for name, fn in (("one", one), ("two", two), ("three", three)):
        res[name].append(timed(fn))
assert torch.equal(mixed, ref)
print(json.dumps({"experiment": "tools/probe/two_stream.py", "us_per_mix_median": {k: round(statistics.median(v), 2) for k, v in res.items()},
                  "us_per_mix_min": {k: round(min(v), 2) for k, v in res.items()}}))
