"""Placement-calibrated allocation of a population's bucket stacks.

The same streaming mix runs at one of a few discrete rates depending on the device memory its
buffers land on (about 156-168 us per K = 8 x 25M mix on MI355X, DESIGN.md §3 "Placement
variance"). The level is a property of each allocation, fixed for its lifetime: of the stack the
mixes read, or of the stack they write (``tools/probe/placement_pairs.py``). No allocation method
controls it: torch's allocator, hipExtMalloc default / contiguous / fine-grained / uncached, and
virtual-memory mappings backed by 2 MiB, 64 MiB, 1 GiB or whole-range physical handles at 1 GiB
aligned addresses all spread over the same levels (``tools/alloc_experiment.py``,
``tools/probe/vmm_placement.py``). Large allocations tend to the fast level
(``tools/probe/alloc_size.py``), so candidate stacks are carved from allocations of 16 GiB or
more.

A population lives for the whole run, so it can afford to choose: ``calibrated_stacks`` allocates
``candidates`` input stacks and as many output stacks (HBM holds them: the bench population is
26 GB of 288), times the population's own ring-window mix on a spread of rows of each, keeps the
fastest output stack (against the first input), then the fastest input stack with it, then the
output again with that input, and drops the others into torch's caching allocator (returning
them to the driver is an option: the driver's background scrub of freed memory then costs a
settle period). The probe runs the production kernel on the stacks as they will be used; it
changes where the buckets live, not what is computed."""
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


def spare_view(stack: torch.Tensor, shapes, align: int = 64) -> Optional[List[torch.Tensor]]:
    """Views of the given ``shapes`` carved, in order and ``align``-element aligned, from the part
    of ``stack``'s allocation that lies past the stack itself (a calibrated stack is the head of
    an allocation of 16 GiB or more, ``calibrated_stacks``), or None when the allocation has no
    room. The shard's halo rows and relay slots live there, on the calibrated allocation instead
    of small allocations of their own (which tend to land on the slower placement level)."""
    st = stack.untyped_storage()
    esize = stack.element_size()
    total = st.nbytes() // esize
    off = stack.storage_offset() + stack.numel()
    views = []
    for shape in shapes:
        n = 1
        for x in shape:
            n *= int(x)
        off = -(-off // align) * align
        if off + n > total:
            return None
        views.append(torch.empty(0, dtype=stack.dtype, device=stack.device).set_(st, off, tuple(shape)))
        off += n
    return views


def fit_candidates(candidates: int, stack_bytes: int, free_bytes: int, budget_frac: float) -> int:
    """How many (input, output) candidate pairs of ``stack_bytes`` allocations the probe may hold
    at once within ``budget_frac`` of ``free_bytes`` (at least one: the plain allocation)."""
    return max(1, min(int(candidates), int(budget_frac * free_bytes) // max(1, 2 * int(stack_bytes))))


def calibrated_stacks(L: int, P: int, device, engine, hl: int, hr: int, candidates: int = 4,
                      rows: int = 128, passes: int = 3, dtype=torch.float32,
                      timer: Optional[Callable] = None, hold: Optional[list] = None,
                      settle_s: float = 8.0, release: bool = False,
                      min_alloc_bytes: int = 16 << 30, budget_frac: float = 0.6
                      ) -> Tuple[torch.Tensor, torch.Tensor, dict]:
    """(models, mixed, report): two ``[L, P]`` stacks chosen among ``candidates`` allocations each
    (output, then input, then output again) by timing the ring-window sequential mix (``hl``
    below, ``hr`` above, wrap-around within the stack) of ``rows`` spread rows. ``report`` holds
    every candidate's median microseconds per mix and the chosen indices. ``timer(fns) ->
    seconds`` replaces the HIP-event timing (tests). ``hold``: a list that receives the rejected
    candidates instead of dropping them (measurement of their effect). Dropped candidates stay in
    torch's caching allocator, reusable by the process's later allocations, as any freed tensor
    does. ``release=True`` returns them to the driver instead (``torch.cuda.empty_cache``); the
    driver then scrubs that memory in the background, which slows every mix by 1-3% for a few
    seconds, so mixes run on the chosen pair until their rate has settled (at most ``settle_s``
    seconds; ``report["settle"]``). Each candidate stack is carved from an allocation of at
    least ``min_alloc_bytes`` (device stacks of 1 GiB or more): a 16-device ring mixed from 16-, 32- or 64-row
    allocations ran at 161-164 us, from the first 16 rows of a 128-row (12.8 GB) allocation at
    154 us, in either allocation order (tools/probe/alloc_size.py).

    Footprint: the probe holds 2 x ``candidates`` such allocations at once, so ``candidates`` is
    capped to what fits in ``budget_frac`` of the device's free memory at entry. The chosen pair
    keeps its whole allocations alive (the placement is a property of the allocation). The report
    states the allocation size, the bytes the chosen pair holds, the bytes the rejected candidates
    leave in torch's cache (0 with ``release``), and ``plain_us``: the probe time of candidate
    pair (0, 0), the first allocation of each stack, i.e. what the population runs at without the
    choice."""
    if candidates < 1:
        raise ValueError("need at least one candidate")
    if candidates > 1 and engine is None:
        raise ValueError("the placement probe needs an engine (the mix it times)")
    dev = torch.device(device)
    ins, outs = [], []
    esize = dtype.itemsize
    big = dev.type == "cuda" and L * P * esize >= (1 << 30)  # streaming-bound stacks only
    floor = max(L * P, (min_alloc_bytes // esize) if big else 0)

    def stack():
        base = torch.empty(floor, dtype=dtype, device=dev)
        return base[:L * P].view(L, P)

    capped = None
    if dev.type == "cuda" and candidates > 1:
        fit = fit_candidates(candidates, floor * esize, torch.cuda.mem_get_info(dev)[0], budget_frac)
        if fit < candidates:
            capped, candidates = candidates, fit

    for c in range(candidates):  # as many pairs as fit: never fail where a plain allocation would not
        try:
            pair = (stack(), stack())
        except torch.OutOfMemoryError:
            if not ins:
                raise
            break
        ins.append(pair[0])
        outs.append(pair[1])
    candidates = len(ins)
    gib = float(1 << 30)
    footprint = {"alloc_GiB_per_stack": round(floor * esize / gib, 3),
                 "data_GiB_per_stack": round(L * P * esize / gib, 3)}
    if capped is not None:
        footprint["candidates_capped_from"] = capped
    if candidates == 1:
        return ins[0], outs[0], {"candidates": 1, **footprint}
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

    gen = torch.Generator(device=dev).manual_seed(20261015)
    for m in ins:  # finite values like the population's own (zeros run 0.3-0.6% faster)
        m.normal_(generator=gen)
    # coordinate descent: a slow stack on one side masks the other side's differences, so the
    # output is chosen against input 0, the input against that output, then the output again
    t_out0 = measure([plan(ins[0], o) for o in outs])
    b = choose(t_out0)
    t_in = measure([plan(m, outs[b]) for m in ins])
    a = choose(t_in)
    t_out = measure([plan(ins[a], o) for o in outs]) if a != 0 else t_out0
    b = choose(t_out)
    models, mixed = ins[a], outs[b]
    if hold is not None:
        hold.extend(t for i, t in enumerate(ins) if i != a)
        hold.extend(t for j, t in enumerate(outs) if j != b)
    del ins, outs
    settle = None
    if dev.type == "cuda" and release:
        torch.cuda.empty_cache()
        if timer is None and settle_s > 0:
            target = statistics.median(t_out[b])
            settle = _settle(plan(models, mixed), run_time, target, settle_s)
    report = {"candidates": candidates, "probe_rows": len(sel),
              "out_us_vs_in0": [round(statistics.median(t), 2) for t in t_out0],
              "in_us": [round(statistics.median(t), 2) for t in t_in],
              "out_us": [round(statistics.median(t), 2) for t in t_out], "chosen": [a, b],
              "plain_us": round(statistics.median(t_out0[0]), 2),
              "chosen_us": round(statistics.median(t_out[b]), 2),
              **footprint,
              "held_GiB": round(2 * floor * esize / gib, 3),
              "rejected_cached_GiB": 0.0 if release else round((2 * candidates - 2) * floor * esize / gib, 3)}
    if settle is not None:
        report["settle"] = settle
    return models, mixed, report


def _settle(fns, run_time, target_us: float, max_s: float, window: int = 5, tol: float = 0.006) -> dict:
    """Mixes on the chosen pair until two windows' medians in a row are back within ``tol`` of what
    the pair ran at in the probe (``target_us``), or ``max_s`` seconds pass. Freeing the rejected
    candidates slows every mix by 1-3% for a few seconds (the freed memory is evidently scrubbed
    in the background: the rate steps back up about 3 s after 77 GB are freed,
    tools/probe/placement_followup.py), so the caller's first timed rounds would otherwise run
    inside that transient."""
    import time
    t0, meds, ok = time.perf_counter(), [], 0
    while True:
        med = statistics.median(run_time(fns) / len(fns) * 1e6 for _ in range(window))
        meds.append(round(med, 2))
        ok = ok + 1 if med <= target_us * (1.0 + tol) else 0
        done = ok >= 2  # two windows in a row: one can dip under while the scrub still runs
        if done or time.perf_counter() - t0 > max_s:
            return {"seconds": round(time.perf_counter() - t0, 2), "target_us": round(target_us, 2),
                    "window_medians_us": meds, "settled": bool(done)}


def calibrated_rotation(count: int, L: int, P: int, device, engine, candidates: int = 6, hl: int = 2,
                        hr: int = 2, rows: int = 64, passes: int = 3, dtype=torch.float32,
                        timer: Optional[Callable] = None, min_alloc_bytes: int = 16 << 30,
                        budget_frac: float = 0.6) -> Tuple[List[torch.Tensor], dict]:
    """``count`` ``[L, P]`` stacks for a population whose rounds ROTATE its stacks through every
    role (read as the current models, read as the previous round's published models, written as
    the output: ``topology.Tf1PopulationRound``'s (current, previous, out), cfa.py:105-154), chosen
    among ``candidates`` allocations (each carved from ``min_alloc_bytes`` or more, as in
    ``calibrated_stacks``).

    Every stack is both read and written over a rotation, so each candidate is scored by the sum
    of two median probe times: written as the output of a ring-window sequential mix (``hl``
    below, ``hr`` above) of ``rows`` spread rows whose inputs are two other candidates, and read as
    the current models with the same two others as neighbours and output. The ``count`` lowest
    scores are kept (ties to the earlier candidate); the rest go to torch's cache. Returns (stacks
    in candidate order, report with every score and ``plain_us``: the score of candidates
    0..count-1, the stacks a plain allocation gets)."""
    if count < 1:
        raise ValueError("need at least one stack")
    dev = torch.device(device)
    esize = dtype.itemsize
    big = dev.type == "cuda" and L * P * esize >= (1 << 30)
    floor = max(L * P, (min_alloc_bytes // esize) if big else 0)
    if candidates > count and dev.type == "cuda":
        fit = int(budget_frac * torch.cuda.mem_get_info(dev)[0]) // max(1, floor * esize)
        candidates = max(count, min(candidates, fit))
    if candidates <= count or L < 1:
        stacks = [torch.zeros(L, P, dtype=dtype, device=dev) for _ in range(count)]
        return stacks, {"candidates": count}
    if engine is None:
        raise ValueError("the placement probe needs an engine (the mix it times)")
    cand = []
    for _ in range(candidates):
        try:
            cand.append(torch.empty(floor, dtype=dtype, device=dev)[:L * P].view(L, P))
        except torch.OutOfMemoryError:
            break
    if len(cand) <= count:
        return cand[:count] + [torch.zeros(L, P, dtype=dtype, device=dev) for _ in range(count - len(cand))], \
            {"candidates": len(cand)}
    gen = torch.Generator(device=dev).manual_seed(20261015)
    for c in cand:
        c.normal_(generator=gen)
    K = hl + hr
    alphas = [1.0 / (K + 1)] * K
    offsets = [o for o in range(-hl, 0)] + [o for o in range(1, hr + 1)]
    sel = probe_rows(L, rows)

    def plan(cur, prev, out):
        return [engine.prepare_mix_seq(out[d], cur[d], [prev[(d + k) % L] for k in offsets], alphas) for d in sel]

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

    def others(c):
        o = [i for i in range(len(cand)) if i != c]
        return o[0], o[1]

    plans = []
    for c in range(len(cand)):
        a, b = others(c)
        plans.append(plan(cand[a], cand[b], cand[c]))  # c written
        plans.append(plan(cand[c], cand[a], cand[b]))  # c read as the current models
    for fns in plans:
        run_time(fns)
    t = [[] for _ in plans]
    for _ in range(passes):
        for i, fns in enumerate(plans):
            t[i].append(run_time(fns) / len(fns) * 1e6)
    out_us = [statistics.median(t[2 * c]) for c in range(len(cand))]
    in_us = [statistics.median(t[2 * c + 1]) for c in range(len(cand))]
    score = [o + i for o, i in zip(out_us, in_us)]
    keep = sorted(sorted(range(len(cand)), key=lambda c: (score[c], c))[:count])
    chosen = [cand[c] for c in keep]
    del cand, plans
    gib = float(1 << 30)
    report = {"candidates": len(score), "probe_rows": len(sel), "out_us": [round(x, 2) for x in out_us],
              "in_us": [round(x, 2) for x in in_us], "chosen": keep,
              "plain_us": round(statistics.mean(score[:count]) / 2, 2),
              "chosen_us": round(statistics.mean(score[c] for c in keep) / 2, 2),
              "alloc_GiB_per_stack": round(floor * esize / gib, 3), "data_GiB_per_stack": round(L * P * esize / gib, 3),
              "rejected_cached_GiB": round((len(score) - count) * floor * esize / gib, 3)}
    return chosen, report
