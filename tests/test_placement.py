"""Host logic of the placement-calibrated stacks (federated_amd/placement.py): probe rows, the
choice rule, and that calibrated_stacks keeps the fastest input stack, then the fastest output
stack with it (stub engine and timer on CPU tensors)."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from federated_amd import placement  # noqa: E402
from federated_amd.population import make_ring_shard  # noqa: E402


def test_probe_rows_spread_and_small_stacks():
    assert placement.probe_rows(128, 8) == [0, 16, 32, 48, 64, 80, 96, 112]
    assert placement.probe_rows(5, 8) == [0, 1, 2, 3, 4]
    assert placement.probe_rows(9, 8) == sorted(set(placement.probe_rows(9, 8)))


def test_choose_takes_the_smallest_median_first_on_ties():
    assert placement.choose([[5, 5, 9], [4, 4, 6], [7, 1, 7]]) == 1
    assert placement.choose([[3.0], [3.0]]) == 0


class StubEngine:
    """prepare_mix_seq returns a launch tagged with the (local, out) stacks it touches."""

    def __init__(self):
        self.calls = []

    def prepare_mix_seq(self, out, local, nbrs, alphas):
        assert len(nbrs) == len(alphas)

        def launch(stream=None):
            pass

        launch.tag = (local.untyped_storage().data_ptr(), out.untyped_storage().data_ptr())
        return launch


@pytest.mark.parametrize("slow_in,slow_out", [({0: 9.0, 2: 7.0}, {1: 8.0}), ({}, {0: 3.0, 3: 3.0})])
def test_calibrated_stacks_keep_the_fastest_input_then_output(monkeypatch, slow_in, slow_out):
    C, L, P = 4, 6, 32
    made = []
    real_empty = torch.empty

    def tracking_empty(*a, **k):
        t = real_empty(*a, **k)
        made.append(t)
        return t

    monkeypatch.setattr(placement.torch, "empty", tracking_empty)
    cost = {}

    def timer(fns):
        ins = [t.untyped_storage().data_ptr() for t in made[0:2 * C:2]]  # allocated in (input, output) pairs
        outs = [t.untyped_storage().data_ptr() for t in made[1:2 * C:2]]
        i_ptr, o_ptr = fns[0].tag
        i, o = ins.index(i_ptr), outs.index(o_ptr)
        return len(fns) * 1e-6 * (1.0 + slow_in.get(i, 0.0) + slow_out.get(o, 0.0))

    models, mixed, rep = placement.calibrated_stacks(L, P, "cpu", StubEngine(), 2, 2, candidates=C, rows=3,
                                                     timer=timer)
    a = min(range(C), key=lambda i: (slow_in.get(i, 0.0), i))
    b = min(range(C), key=lambda j: (slow_out.get(j, 0.0), j))
    assert rep["chosen"] == [a, b]
    assert models.untyped_storage().data_ptr() == made[2 * a].untyped_storage().data_ptr()
    assert mixed.untyped_storage().data_ptr() == made[2 * b + 1].untyped_storage().data_ptr()
    assert tuple(models.shape) == (L, P) and tuple(mixed.shape) == (L, P)
    assert len(rep["in_us"]) == C and len(rep["out_us"]) == C and rep["probe_rows"] == 3
    assert bool(torch.all(torch.isfinite(models)))  # probed on finite values
    # pair (0, 0) is the plain-allocation figure; the chosen pair's time is never above it
    assert rep["plain_us"] == rep["out_us_vs_in0"][0]
    assert rep["chosen_us"] <= rep["plain_us"]
    gib = L * P * 4 / float(1 << 30)
    assert rep["held_GiB"] == round(2 * gib, 3)
    assert rep["rejected_cached_GiB"] == round((2 * C - 2) * gib, 3)


def test_probe_footprint_is_capped_by_free_memory():
    """The probe holds 2 x candidates allocations: never more than budget_frac of free memory."""
    GiB = 1 << 30
    assert placement.fit_candidates(4, 16 * GiB, 288 * GiB, 0.6) == 4   # the bench: 128 of 172 GiB
    assert placement.fit_candidates(4, 16 * GiB, 100 * GiB, 0.6) == 1   # 60 GiB holds one pair
    assert placement.fit_candidates(4, 16 * GiB, 120 * GiB, 0.6) == 2
    assert placement.fit_candidates(4, 16 * GiB, 10 * GiB, 0.6) == 1    # never below the plain pair


def test_one_candidate_is_a_plain_allocation():
    m, o, rep = placement.calibrated_stacks(3, 8, "cpu", None, 1, 1, candidates=1)
    assert rep["candidates"] == 1 and tuple(m.shape) == (3, 8) and tuple(o.shape) == (3, 8)
    assert rep["data_GiB_per_stack"] == rep["alloc_GiB_per_stack"]  # host stacks: no floor


def test_ring_shard_takes_caller_stacks_and_checks_them():
    from federated_amd.population import RingPopulationShard, RingShardPlan
    plan = RingShardPlan(0, 1, 4, 1)
    m, o = torch.zeros(4, 16), torch.zeros(4, 16)
    shard = RingPopulationShard(plan, 16, "cpu", stacks=(m, o))
    assert shard.models is m and shard.mixed is o
    with pytest.raises(ValueError):
        RingPopulationShard(plan, 16, "cpu", stacks=(torch.zeros(3, 16), o))
    # on CPU (no HIP engine) make_ring_shard skips the calibration and says so
    _, info = make_ring_shard(0, 1, 4, 1, 1, 16, "cpu", placement_candidates=4)
    assert info["placement"] is None


def test_calibration_uses_the_pairs_that_fit(monkeypatch):
    """Out of memory after two candidate pairs: the probe runs on those two instead of failing."""
    real_empty, n = torch.empty, [0]

    def limited_empty(*a, **k):
        n[0] += 1
        if n[0] > 4:
            raise torch.OutOfMemoryError("stub: out of memory")
        return real_empty(*a, **k)

    monkeypatch.setattr(placement.torch, "empty", limited_empty)
    m, o, rep = placement.calibrated_stacks(4, 16, "cpu", StubEngine(), 1, 1, candidates=4, rows=2,
                                            timer=lambda fns: 1e-6 * len(fns))
    assert rep["candidates"] == 2 and rep["chosen"] == [0, 0] and tuple(m.shape) == (4, 16)


def test_probe_without_engine_is_refused():
    with pytest.raises(ValueError):
        placement.calibrated_stacks(4, 16, "cpu", None, 1, 1, candidates=2)


def test_calibrated_rotation_drops_the_slow_candidates():
    """Rotating stacks (Tf1PopulationRound): a candidate slow as output and as input is dropped;
    the kept stacks are the lowest scores in candidate order."""
    C, L, P = 6, 5, 16
    slow = {1: 5.0, 4: 5.0}
    made = []

    class TagEngine(StubEngine):
        def prepare_mix_seq(self, out, local, nbrs, alphas):
            fn = super().prepare_mix_seq(out, local, nbrs, alphas)
            made.append(fn)
            return fn

    stacks_holder = {}

    def timer(fns):
        ptrs = stacks_holder["ptrs"]
        i_ptr, o_ptr = fns[0].tag
        return len(fns) * 1e-6 * (1.0 + slow.get(ptrs.index(o_ptr), 0.0) + slow.get(ptrs.index(i_ptr), 0.0))

    real_empty = torch.empty
    allocs = []

    def tracking_empty(*a, **k):
        t = real_empty(*a, **k)
        allocs.append(t)
        stacks_holder["ptrs"] = [x.untyped_storage().data_ptr() for x in allocs]
        return t

    import unittest.mock as um
    with um.patch.object(placement.torch, "empty", tracking_empty):
        stacks, rep = placement.calibrated_rotation(3, L, P, "cpu", TagEngine(), candidates=C, rows=3, timer=timer)
    assert rep["candidates"] == C and len(stacks) == 3
    assert 1 not in rep["chosen"] and 4 not in rep["chosen"]
    assert rep["chosen"] == sorted(rep["chosen"])
    assert [s.untyped_storage().data_ptr() for s in stacks] == [stacks_holder["ptrs"][c] for c in rep["chosen"]]
    assert all(tuple(s.shape) == (L, P) for s in stacks)
    assert rep["chosen_us"] <= rep["plain_us"]


def test_calibrated_rotation_plain_when_no_spare_candidates():
    stacks, rep = placement.calibrated_rotation(3, 4, 8, "cpu", None, candidates=3)
    assert rep == {"candidates": 3} and len(stacks) == 3 and all(float(s.abs().sum()) == 0 for s in stacks)


def test_spare_view_carves_after_the_stack():
    base = torch.arange(1000, dtype=torch.float32)
    stack = base[:2 * 100].view(2, 100)
    v = placement.spare_view(stack, [(3, 50), (2, 7)], align=64)
    assert v is not None and tuple(v[0].shape) == (3, 50) and tuple(v[1].shape) == (2, 7)
    assert v[0].storage_offset() == 256 and v[1].storage_offset() == 448  # 64-aligned after 200
    assert float(v[0][0, 0]) == 256.0
    v[1].fill_(-1)
    assert float(base[448]) == -1 and float(base[461]) == -1 and float(base[462]) == 462
    assert placement.spare_view(stack, [(9, 100)]) is None  # no room
    assert placement.spare_view(torch.zeros(2, 100), [(1, 1)]) is None  # a plain stack has none


def test_ring_shard_halo_and_relay_carved_from_calibrated_stacks():
    """World 8 shard on caller stacks with spare room: halo rows and relay slots live in the
    models allocation past the stack, and the routed exchange uses them."""
    from federated_amd.halo import RoutePlan, ring_transfers
    from federated_amd.population import RingPopulationShard, RingShardPlan
    L, P, h, world, rank = 16, 4096, 4, 8, 3
    plan = RingShardPlan(rank, world, L, h)
    route = RoutePlan(world, ring_transfers(world, L, h, h, P))
    big_m = torch.zeros(L * P + 2 * h * P + 2 * route.slot_elems(rank) + 1024)
    m, o = big_m[:L * P].view(L, P), torch.zeros(L, P)
    shard = RingPopulationShard(plan, P, "cpu", stacks=(m, o), route=route, rank=rank, carve=True)
    assert shard.carved
    ptr0, ptr1 = big_m.data_ptr(), big_m.data_ptr() + big_m.numel() * 4
    for t in (shard.halo["left"], shard.halo["right"], shard.routed().relay):
        assert ptr0 + L * P * 4 <= t.data_ptr() < ptr1
    plain = RingPopulationShard(plan, P, "cpu", stacks=(torch.zeros(L, P), o), route=route, rank=rank, carve=True)
    assert not plain.carved and plain.routed().relay.shape[0] == 2
    # caller stacks are not carved unless asked (the spare room may belong to someone else)
    assert not RingPopulationShard(plan, P, "cpu", stacks=(m, o), route=route, rank=rank).carved


def test_ring_shard_refuses_a_carve_over_the_mixed_stack():
    """Stacks cut from ONE caller allocation (models first, mixed right after): the spare room past
    the models stack IS the mixed stack, so a carve would alias it; the shard allocates its halo on
    its own and a round still equals the unsharded oracle."""
    from federated_amd.halo import RoutePlan, ring_transfers
    from federated_amd.population import RingPopulationShard, RingShardPlan
    L, P, h, world, rank = 8, 256, 2, 4, 1
    plan = RingShardPlan(rank, world, L, h)
    route = RoutePlan(world, ring_transfers(world, L, h, h, P))
    buf = torch.zeros(2, L, P)
    shard = RingPopulationShard(plan, P, "cpu", stacks=(buf[0], buf[1]), route=route, rank=rank, carve=True)
    assert not shard.carved
    lo, hi = buf[1].data_ptr(), buf[1].data_ptr() + buf[1].numel() * 4
    for t in (shard.halo["left"], shard.halo["right"]):
        assert not (lo <= t.data_ptr() < hi)


def test_scattered_order_keeps_consecutive_windows_apart():
    from federated_amd.population import scattered_order
    K, L = 8, 128
    order = scattered_order(list(range(L)), K)
    assert sorted(order) == list(range(L))

    def window(g):
        return {(g + o) % L for o in range(-K // 2, K // 2 + 1)}

    for a, b, c in zip(order, order[1:], order[2:]):
        assert not window(c) & (window(a) | window(b))
    assert scattered_order([3, 4], 8) == [3, 4]
