"""The host lane on the GPU (federated_amd/hostlane.py): halo pieces over PCIe through pinned shared
host memory, D2H and H2D ordered across processes by cfa_stream_signal / cfa_stream_wait_word.

- The wait kernel: a word that never comes ends the wait after its timeout with the status word
  set, and every later wait on that status returns at once; a word raised by another stream
  releases it.
- Two processes on the one GPU (the lane's mechanism is per process pair, whichever GPUs they
  drive): the ring population sharded in 2 device blocks, the route planned with equal xGMI and
  lane rates so half the halo takes the lane (the rest over torch.distributed/gloo), several rounds
  with the mixed models fed back, every device bit for bit equal to the unsharded oracle
  trajectory (oracle/cfa_oracle.sequential_mix).
"""
import ctypes
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev_ptr(lib, t):
    from federated_amd import _lib
    dp = ctypes.c_void_p()
    _lib.check("cfa_host_device_pointer", lib.cfa_host_device_pointer(ctypes.c_void_p(t.data_ptr()), ctypes.byref(dp)))
    return dp.value


def test_stream_wait_word_timeout_and_release(gpu):
    from federated_amd import _lib
    lib = _lib.load()
    word = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    status = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    wd, sd = _dev_ptr(lib, word), _dev_ptr(lib, status)
    s = torch.cuda.Stream()
    sh = ctypes.c_void_p(s.cuda_stream)
    t0 = time.monotonic()
    _lib.check("wait", lib.cfa_stream_wait_word(ctypes.c_void_p(wd), 5, 200_000, ctypes.c_void_p(sd), sh))
    _lib.check("wait", lib.cfa_stream_wait_word(ctypes.c_void_p(wd), 7, 20_000_000, ctypes.c_void_p(sd), sh))
    s.synchronize()
    dt = time.monotonic() - t0
    assert int(status[0]) == 5  # the first wait timed out; the second returned at once
    assert 0.15 < dt < 5.0
    # released by a signal on another stream
    status.zero_()
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    _lib.check("wait", lib.cfa_stream_wait_word(ctypes.c_void_p(wd), 9, 10_000_000, ctypes.c_void_p(sd),
                                                ctypes.c_void_p(a.cuda_stream)))
    marker = torch.zeros(1, device="cuda")
    with torch.cuda.stream(a):
        marker.fill_(1.0)  # after the wait on stream a
    _lib.check("signal", lib.cfa_stream_signal(ctypes.c_void_p(wd), 9, ctypes.c_void_p(b.cuda_stream)))
    a.synchronize()
    b.synchronize()
    assert int(status[0]) == 0 and int(word[0]) == 9 and float(marker.item()) == 1.0
    with pytest.raises(RuntimeError):
        _lib.check("wait", lib.cfa_stream_wait_word(ctypes.c_void_p(wd), 1, 0, ctypes.c_void_p(sd), sh))


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
        q.put((rank, out, info["route"]["lane"], info.get("lane")))
        shard.lane.close()
    except Exception as exc:  # reported by the parent
        q.put((rank, f"{type(exc).__name__}: {exc}", None, None))
    finally:
        dist.destroy_process_group()


def test_host_lane_two_processes_match_the_oracle(gpu, monkeypatch):
    import torch.multiprocessing as mp
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")  # as bench.py's ranks (bench.set_hw_queues)
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
