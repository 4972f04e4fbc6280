"""The host lane on the GPU (federated_amd/hostlane.py): halo pieces over PCIe through pinned shared
host memory; the sender's D2H raises a word with cfa_stream_signal, the receiver's host waits for
it (cfa_host_wait_word) and only then enqueues the H2D, so no wait parks on a GPU queue.

- Two processes on the one GPU (the lane's mechanism is per process pair, whichever GPUs they
  drive): the ring population sharded in 2 device blocks, the route planned with equal xGMI and
  lane rates so half the halo takes the lane (the rest over torch.distributed/gloo), several rounds
  with the mixed models fed back, every device bit for bit equal to the unsharded oracle
  trajectory (oracle/cfa_oracle.sequential_mix); run at the box's own GPU_MAX_HW_QUEUES (4 on this
  pool: round 6 no longer raises it).
- A lane round whose peer is late does not hold the compute stream: mixes enqueued before the
  round's receive side complete while the host waits for the peer.
"""
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, D, P, rounds, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from federated_amd.engine import get_engine
        from federated_amd.halo import LANE_IN, LANE_OUT
        from federated_amd.hostlane import new_token
        from federated_amd.linkprobe import agree_gloo
        from federated_amd.population import make_ring_shard
        tok = [new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        rates = {(a, b): 50.0 for a in range(world) for b in range(world) if a != b}
        rates.update({(a, LANE_OUT): 50.0 for a in range(world)})
        rates.update({(LANE_IN, a): 50.0 for a in range(world)})
        eng = get_engine(0)
        shard, info = make_ring_shard(rank, world, D, 4, 4, P, torch.device("cuda", 0), TorchTransport(), eng,
                                      link_rates=rates, lane_token=tok[0], lane_agree=agree_gloo,
                                      lane_chunk_elems=1 << 16)
        plan = shard.plan
        for i in range(plan.L):
            g = plan.first + i
            shard.models[i].copy_(torch.randn(P, generator=torch.Generator().manual_seed(5200 + g)))
        cs, ms = torch.cuda.current_stream(), torch.cuda.Stream()
        for _ in range(rounds):
            shard.round(cs, ms)
            shard.models.copy_(shard.mixed)
        torch.cuda.synchronize()
        shard.lane.check()
        out = {plan.first + i: shard.models[i].cpu().numpy() for i in range(plan.L)}
        info["lane"]["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
        q.put((rank, out, info["route"]["lane"], info.get("lane")))
        shard.lane.close()
    except Exception as exc:  # reported by the parent
        q.put((rank, f"{type(exc).__name__}: {exc}", None, None))
    finally:
        dist.destroy_process_group()


def test_host_lane_two_processes_match_the_oracle(gpu):
    import torch.multiprocessing as mp
    from federated_amd.population import RingShardPlan
    from oracle.cfa_oracle import sequential_mix
    D, P, rounds, world = 16, 300_037, 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34500 + (os.getpid() % 997)
    procs = [ctx.Process(target=_worker, args=(r, world, port, D, P, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in procs:
            rank, out, used_lane, lane_info = q.get(timeout=100)
            assert not isinstance(out, str), f"rank {rank}: {out}"
            assert used_lane and lane_info["in_MB"] > 0 and lane_info["out_MB"] > 0
            assert lane_info["hw_queues"] == os.environ.get("GPU_MAX_HW_QUEUES")  # the box's own setting
            got.update(out)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    ring = RingShardPlan(0, 1, D, 4)
    cur = [torch.randn(P, generator=torch.Generator().manual_seed(5200 + g)).numpy() for g in range(D)]
    alphas = [1.0 / 9] * 8
    for _ in range(rounds):
        cur = [sequential_mix(cur[g], [cur[j] for j in ring.neighbours(g)], alphas) for g in range(D)]
    for g in range(D):
        assert np.array_equal(got[g], cur[g]), g


def _late_peer_worker(rank, port, q, delay_s):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from federated_amd.halo import Message
        from federated_amd.hostlane import HostLane, new_token
        from federated_amd.linkprobe import agree_gloo
        tok = [new_token() if rank == 0 else None]
        dist.broadcast_object_list(tok, src=0)
        n = 1 << 22
        bufs = {"send": torch.full((n,), float(rank + 1), device="cuda"), "recv": torch.zeros(n, device="cuda")}
        msgs = [Message(0, a, 1 - a, "send", 0, "recv", 0, n, lane=True) for a in range(2)]
        lane = HostLane.open(rank, [m for m in msgs if m.src == rank], [m for m in msgs if m.dst == rank],
                             lambda k: bufs[k], torch.device("cuda", 0), tok[0], agree_gloo,
                             chunk_elems=1 << 20, timeout_s=30.0)
        cs = torch.cuda.current_stream()
        x = torch.randn(1 << 24, device="cuda")
        torch.cuda.synchronize()
        out = {}
        if rank == 1:
            time.sleep(delay_s)  # the peer is late: rank 0's receive side has nothing to copy yet
        gates = lane.run(cs)
        # compute enqueued AFTER the round started, on the stream the lane's copies follow: with the
        # receive-side wait on the host, nothing on any GPU queue waits for the late peer
        done = torch.cuda.Event()
        for _ in range(20):
            x.mul_(1.0001)
        done.record(cs)
        if rank == 0:
            t0 = time.monotonic()
            while not done.query() and time.monotonic() - t0 < 0.5 * delay_s:
                time.sleep(0.005)
            out["compute_done_while_peer_late"] = bool(done.query())
            out["peer_arrived_by_then"] = _reached_word(lane)
        cs.wait_event(gates[0])
        lane.wait_streams(cs)
        torch.cuda.synchronize()
        out["rows_ok"] = float(bufs["recv"][0]) == float(2 - rank) and float(bufs["recv"][-1]) == float(2 - rank)
        agree_gloo(True)
        lane.close()
        q.put((rank, out))
    except Exception as exc:
        q.put((rank, f"{type(exc).__name__}: {exc}"))
    finally:
        dist.destroy_process_group()


def _reached_word(lane):
    from federated_amd.hostlane import READY
    return any(seg.read(READY) != 0 for seg in lane.in_seg.values())


def test_late_peer_does_not_hold_the_compute_stream(gpu):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34700 + (os.getpid() % 997)
    procs = [ctx.Process(target=_late_peer_worker, args=(r, port, q, 4.0)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            r, out = q.get(timeout=100)
            assert not isinstance(out, str), f"rank {r}: {out}"
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert res[0]["compute_done_while_peer_late"] and not res[0]["peer_arrived_by_then"]
    assert res[0]["rows_ok"] and res[1]["rows_ok"]


def _fuzz_worker(rank, world, port, cases, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.dist import TorchTransport
        from federated_amd.engine import get_engine
        from federated_amd.halo import LANE_IN, LANE_OUT
        from federated_amd.hostlane import new_token
        from federated_amd.linkprobe import agree_gloo
        from federated_amd.population import make_ring_shard
        from federated_amd.streams import role_stream
        eng = get_engine(0)
        outs = []
        for ci, (D, h, P, chunk, lane_rate, rounds) in enumerate(cases):
            tok = [new_token() if rank == 0 else None]
            dist.broadcast_object_list(tok, src=0)
            rates = {(a, b): 50.0 for a in range(world) for b in range(world) if a != b}
            rates.update({(a, LANE_OUT): lane_rate for a in range(world)})
            rates.update({(LANE_IN, a): lane_rate for a in range(world)})
            shard, info = make_ring_shard(rank, world, D, h, h, P, torch.device("cuda", 0), TorchTransport(), eng,
                                          link_rates=rates, lane_token=tok[0], lane_agree=agree_gloo,
                                          lane_chunk_elems=chunk)
            for i in range(shard.plan.L):
                g = shard.plan.first + i
                shard.models[i].copy_(torch.randn(P, generator=torch.Generator().manual_seed(900 + 17 * g + ci)))
            cs = torch.cuda.current_stream()
            for _ in range(rounds):
                shard.round(cs, role_stream("comm"))
                shard.models.copy_(shard.mixed)
            torch.cuda.synchronize()
            outs.append(({shard.plan.first + i: shard.models[i].cpu().numpy() for i in range(shard.plan.L)},
                         bool(info["route"]["lane"])))
            shard.close()
        q.put((rank, outs))
    except Exception as exc:
        q.put((rank, f"{type(exc).__name__}: {exc}"))
    finally:
        dist.destroy_process_group()


def test_host_lane_random_populations_match_the_oracle(gpu):
    """Four random ring populations (window 1-4 per side, odd bucket lengths, chunk sizes from one
    aligned piece to many per row, lane rates from a sliver of the halo to most of it), two
    processes on the GPU, three rounds with the mixed models fed back, every device bit for bit
    against the unsharded oracle trajectory: the lane's host-side pump under the HIP kernels."""
    import random

    import torch.multiprocessing as mp
    from federated_amd.population import RingShardPlan
    from oracle.cfa_oracle import sequential_mix
    rng = random.Random(20261018)
    world, cases = 2, []
    for _ in range(4):
        h = rng.randint(1, 4)
        cases.append((world * rng.randint(2 * h, 2 * h + 2), h, rng.randint(2_000, 60_000) * 2 + 1,
                      64 * rng.randint(1, 200), rng.choice([20.0, 50.0, 200.0]), 3))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 34900 + (os.getpid() % 997)
    procs = [ctx.Process(target=_fuzz_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in procs:
            rank, out = q.get(timeout=100)
            assert not isinstance(out, str), f"rank {rank}: {out}"
            got[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    used = 0
    for ci, (D, h, P, chunk, lane_rate, rounds) in enumerate(cases):
        ring = RingShardPlan(0, 1, D, h)
        cur = [torch.randn(P, generator=torch.Generator().manual_seed(900 + 17 * g + ci)).numpy() for g in range(D)]
        alphas = [1.0 / (2 * h + 1)] * (2 * h)
        for _ in range(rounds):
            cur = [sequential_mix(cur[g], [cur[j] for j in ring.neighbours(g)], alphas) for g in range(D)]
        mine = {**got[0][ci][0], **got[1][ci][0]}
        used += got[0][ci][1]
        for g in range(D):
            assert np.array_equal(mine[g], cur[g]), (ci, g)
    assert used >= 1
