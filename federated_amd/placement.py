"""Placement-calibrated allocation of a population's bucket stacks.

The same streaming mix runs at one of a few discrete rates depending on the device memory its
buffers land on (about 156-168 us per K = 8 x 25M mix on MI355X, DESIGN.md §3 "Placement
variance"). The level is a property of each allocation, fixed for its lifetime: of the stack the
mixes read, or of the stack they write (``tools/probe/placement_pairs.py``). No allocation method
controls it: torch's allocator, hipExtMalloc default / contiguous / fine-grained / uncached, and
virtual-memory mappings backed by 2 MiB, 64 MiB, 1 GiB or whole-range physical handles at 1 GiB
aligned addresses all spread over the same levels (``tools/alloc_experiment.py``,
``tools/probe/vmm_placement.py``).

A population lives for the whole run, so it can afford to choose: ``calibrated_stacks`` allocates
``candidates`` input stacks and as many output stacks (HBM holds them: the bench population is
26 GB of 288), times the population's own ring-window mix on a spread of rows of each, keeps the
fastest output stack (against the first input), then the fastest input stack with it, then the
output again with that input, and frees the others. The probe runs the production kernel on the
stacks as they will be used; it changes where the buckets live, not what is computed."""
from __future__ import annotations

import statistics
from typing import Callable, List, Optional, Sequence, Tuple

import torch


def probe_rows(L: int, count: int) -> List[int]:
    """``count`` device rows spread evenly over ``[0, L)`` (all of them when L <= count)."""
    if L <= count:
        return list(range(L))
    return sorted({(i * L) // count for i in range(count)})


def choose(times: Sequence[Sequence[float]]) -> int:
    """Index of the candidate with the smallest median time (first on ties)."""
    med = [statistics.median(t) for t in times]
    return min(range(len(med)), key=lambda i: (med[i], i))


def calibrated_stacks(L: int, P: int, device, engine, hl: int, hr: int, candidates: int = 4,
                      rows: int = 8, passes: int = 3, dtype=torch.float32,
                      timer: Optional[Callable] = None) -> Tuple[torch.Tensor, torch.Tensor, dict]:
    """(models, mixed, report): two ``[L, P]`` stacks chosen among ``candidates`` allocations each
    (output, then input, then output again) by timing the ring-window sequential mix (``hl``
    below, ``hr`` above, wrap-around within the stack) of ``rows`` spread rows. ``report`` holds
    every candidate's median microseconds per mix and the chosen indices. ``timer(fns) ->
    seconds`` replaces the HIP-event timing (tests)."""
    if candidates < 1:
        raise ValueError("need at least one candidate")
    dev = torch.device(device)
    ins = [torch.empty((L, P), dtype=dtype, device=dev) for _ in range(candidates)]
    outs = [torch.empty((L, P), dtype=dtype, device=dev) for _ in range(candidates)]
    if candidates == 1:
        return ins[0], outs[0], {"candidates": 1}
    K = hl + hr
    alphas = [1.0 / (K + 1)] * K
    offsets = [o for o in range(-hl, 0)] + [o for o in range(1, hr + 1)]
    sel = probe_rows(L, rows)

    def plan(m, o):
        return [engine.prepare_mix_seq(o[d], m[d], [m[(d + k) % L] for k in offsets], alphas) for d in sel]

    def run_time(fns) -> float:
        if timer is not None:
            return timer(fns)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for fn in fns:
            fn(None)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3

    def measure(plans) -> List[List[float]]:
        for fns in plans:  # first touch of every candidate before anything is timed
            run_time(fns)
        t = [[] for _ in plans]
        for _ in range(passes):  # interleaved, so drift affects every candidate alike
            for i, fns in enumerate(plans):
                t[i].append(run_time(fns) / len(fns) * 1e6)
        return t

    for m in ins:  # finite values: the probe's arithmetic must not depend on stale memory
        m.zero_()
    # coordinate descent: a slow stack on one side masks the other side's differences, so the
    # output is chosen against input 0, the input against that output, then the output again
    t_out0 = measure([plan(ins[0], o) for o in outs])
    b = choose(t_out0)
    t_in = measure([plan(m, outs[b]) for m in ins])
    a = choose(t_in)
    t_out = measure([plan(ins[a], o) for o in outs]) if a != 0 else t_out0
    b = choose(t_out)
    models, mixed = ins[a], outs[b]
    del ins, outs
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    report = {"candidates": candidates, "probe_rows": len(sel),
              "out_us_vs_in0": [round(statistics.median(t), 2) for t in t_out0],
              "in_us": [round(statistics.median(t), 2) for t in t_in],
              "out_us": [round(statistics.median(t), 2) for t in t_out], "chosen": [a, b]}
    return models, mixed, report
