"""CPU tests (gloo, world size 2) of the RCCL transport's setup and of the bench's fail-loud rule.

``RcclTransport`` (federated_amd/dist.py) has rank 0 create the RCCL unique id and broadcast it
over the torch.distributed group; every rank then calls ``cfa_comm_init`` with it. Here libcfa's
``call`` is replaced by a stub in each rank process, so the broadcast, the argument plumbing and
the error paths run without a GPU:

- success: every rank initialises its communicator with the same 128 id bytes, its own rank, the
  world size and its device;
- rank 0 cannot create the id: it still broadcasts (the failure), so no rank waits forever, and
  every rank raises;
- ``bench.open_transport``: when any rank fails to open RCCL, EVERY rank raises
  ``TransportError`` (the bench exits non-zero), unless ``allow_fallback``, where every rank takes
  the same torch transport and the line is marked non-comparable; ``--transport torch`` on the
  gloo group is host-staged and marked non-comparable too.
"""
import os
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_lib(rank, fail_uid=False, fail_init_rank=None, log=None):
    """Replace _lib.call in this process: records (name, args) and fills the unique id."""
    import ctypes
    from federated_amd import _lib

    def call(name, *args):
        if name == "cfa_comm_unique_id":
            if fail_uid:
                raise _lib.CFAError(name, _lib.CFA_E_RCCL, "ncclGetUniqueId: stub failure")
            ctypes.memmove(args[0], bytes(range(_lib.CFA_UNIQUE_ID_BYTES)), _lib.CFA_UNIQUE_ID_BYTES)
            return
        if name == "cfa_comm_init":
            comm_p, r, world, uid, device = args
            if fail_init_rank == rank:
                raise _lib.CFAError(name, _lib.CFA_E_RCCL, "ncclCommInitRank: stub failure")
            log.append(("init", r, world, ctypes.string_at(uid, _lib.CFA_UNIQUE_ID_BYTES), device))
            comm_p._obj.value = 0x1000 + r
            return
        if name == "cfa_comm_destroy":
            log.append(("destroy", getattr(args[0], "value", args[0])))
            return
        raise AssertionError(f"unexpected libcfa call {name}")

    _lib.call = call


def _worker(rank, world, port, scenario, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []
    try:
        if scenario == "ok":
            _stub_lib(rank, log=log)
            from federated_amd.dist import RcclTransport
            t = RcclTransport(rank, world, device=rank)
            t.close()
            q.put((rank, "ok", log))
        elif scenario == "uid_fails":
            _stub_lib(rank, fail_uid=True, log=log)
            from federated_amd.dist import RcclTransport
            try:
                RcclTransport(rank, world, device=rank)
                q.put((rank, "no error", log))
            except RuntimeError as exc:
                q.put((rank, "raised: " + str(exc), log))
        elif scenario in ("init_fails", "init_fails_fallback"):
            _stub_lib(rank, fail_init_rank=1, log=log)
            import bench
            try:
                t, comparable = bench.open_transport("rccl", rank, world, rank,
                                                     allow_fallback=scenario.endswith("fallback"))
                q.put((rank, f"opened {t.name} comparable={comparable}", log))
            except bench.TransportError as exc:
                q.put((rank, "TransportError: " + str(exc), log))
        elif scenario == "torch_gloo":
            import bench
            t, comparable = bench.open_transport("torch", rank, world, rank)
            q.put((rank, f"opened {t.name} comparable={comparable}", log))
    finally:
        dist.destroy_process_group()


def _run(scenario, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33000 + (os.getpid() % 911) + 7 * len(scenario)
    procs = [ctx.Process(target=_worker, args=(r, world, port, scenario, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, status, log = q.get(timeout=180)
        res[r] = (status, log)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_rccl_unique_id_broadcast_and_init_args():
    res = _run("ok")
    uid = bytes(range(128))
    for r in (0, 1):
        status, log = res[r]
        assert status == "ok"
        assert log[0] == ("init", r, 2, uid, r)  # same id on every rank, own rank and device
        assert log[1] == ("destroy", 0x1000 + r)


def test_rccl_unique_id_failure_on_rank0_reaches_every_rank():
    res = _run("uid_fails")
    for r in (0, 1):
        status, log = res[r]
        assert status.startswith("raised: RCCL unique id unavailable"), status
        assert "stub failure" in status
        assert log == []  # nobody initialised a communicator with a bogus id


def test_bench_transport_failure_is_fatal_on_every_rank():
    res = _run("init_fails")
    for r in (0, 1):
        status, log = res[r]
        assert status.startswith("TransportError: the rccl transport could not be opened"), status
    assert "stub failure" in res[1][0]
    # the rank whose init succeeded released its communicator before raising
    assert [e[0] for e in res[0][1]] == ["init", "destroy"]


def test_bench_fallback_is_marked_non_comparable():
    res = _run("init_fails_fallback")
    statuses = {res[r][0] for r in (0, 1)}
    assert len(statuses) == 1  # every rank took the same transport
    status = statuses.pop()
    assert status.startswith("opened torch-") and status.endswith("comparable=False"), status


def test_bench_torch_transport_on_gloo_is_not_comparable():
    """``--transport torch`` on the bench's gloo control group stages every exchange through host
    memory: the line must say so."""
    res = _run("torch_gloo")
    for r in (0, 1):
        assert res[r][0] == "opened torch-gloo comparable=False", res[r][0]
