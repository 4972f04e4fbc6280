"""CPU test of libcfa's RCCL transport against a recording RCCL stub.

``federated_amd/csrc/cfa_comm.cpp`` (the product source, unchanged) is compiled here with g++
against test doubles of the RCCL / HIP API subset it uses (``tests/native/rccl_stub``), which log
every ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd per communicator. The Python side is the
product path too: ``dist.RcclTransport.prepare`` builds the ctypes tables and
``halo.RoutedExchange`` issues the groups, for all 8 ranks of the bench's own strong-scaling plan
(D = 128 devices, K = 8 ring window, relayed + staged halo). The test asserts

- per rank and per group: one start, the plan's sends (``RoutePlan.rank_ops``) in order with
  their peers, counts and buffer addresses, then its receives likewise, then one end;
- across ranks: in every group, the k-th send from a to b and the k-th receive on b from a have
  the same length (RCCL pairs point-to-point operations between a rank pair in issue order);
- and, replaying the recorded messages group by group as memory copies, every rank's halo ends
  up holding exactly the neighbour buckets its boundary devices read.

RCCL itself never runs at world > 1 on a one-GPU box; this pins what libcfa hands it.
"""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd.dist import RcclTransport
from federated_amd.population import make_ring_shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "native", "rccl_stub")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("commstub") / "libcommstub.so")
    subprocess.run(["g++", "-std=c++17", "-O1", "-fPIC", "-shared", "-Wall", f"-I{STUB}",
                    f"-I{os.path.join(ROOT, 'include')}", os.path.join(ROOT, "federated_amd", "csrc", "cfa_comm.cpp"),
                    os.path.join(STUB, "rccl_stub.cpp"), "-o", so], check=True, capture_output=True, text=True)
    lib = ctypes.CDLL(so)
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name) and name.startswith(("cfa_comm", "cfa_p2p", "cfa_halo", "cfa_allreduce",
                                                   "cfa_reduce", "cfa_rccl")):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    lib.stub_log.restype, lib.stub_log.argtypes = ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
    lib.stub_last_error.restype = ctypes.c_char_p
    return lib


class StubLib:
    """The ``_lib`` module as RcclTransport sees it, with ``call`` bound to the stub build."""

    def __init__(self, lib):
        self.lib = lib

    def __getattr__(self, name):
        return getattr(_lib, name)

    def call(self, name, *args):
        rc = getattr(self.lib, name)(*args)
        if rc != 0:
            raise _lib.CFAError(name, rc, self.lib.stub_last_error().decode())


def stub_transport(lib, rank, world):
    t = object.__new__(RcclTransport)  # RcclTransport.__init__ broadcasts the id over torch.distributed
    t._lib = StubLib(lib)
    uid = (ctypes.c_char * _lib.CFA_UNIQUE_ID_BYTES)()
    t._lib.call("cfa_comm_unique_id", ctypes.cast(uid, ctypes.c_void_p))
    comm = ctypes.c_void_p()
    t._lib.call("cfa_comm_init", ctypes.byref(comm), rank, world, ctypes.cast(uid, ctypes.c_void_p), 0)
    t.comm, t.rank, t.world, t.device = comm, rank, world, 0
    return t


class DeviceView:
    """A host tensor slice presented as the device buffer RcclTransport.prepare expects (the stub
    never dereferences it)."""

    def __init__(self, t):
        self.t, self.is_cuda, self.dtype = t, True, t.dtype

    def is_contiguous(self):
        return self.t.is_contiguous()

    def numel(self):
        return self.t.numel()

    def data_ptr(self):
        return self.t.data_ptr()


class ViaRccl:
    """The transport RoutedExchange binds: RcclTransport.prepare on the host views."""

    def __init__(self, rccl):
        self.rccl = rccl

    def prepare(self, sends, recvs):
        return self.rccl.prepare([(DeviceView(b), p) for b, p in sends], [(DeviceView(b), p) for b, p in recvs])


class FakeStream:
    def __init__(self, handle):
        self.cuda_stream = handle


def parse(log):
    groups, cur = [], None
    for line in log.splitlines():
        w = line.split()
        if w[0] == "start":
            cur = []
        elif w[0] == "end":
            groups.append(cur)
            cur = None
        else:
            cur.append((w[0], int(w[1]), int(w[2]), int(w[3]), int(w[4])))
    assert cur is None, "group left open"
    return groups


def read_log(lib, comm):
    n = lib.stub_log(comm, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.stub_log(comm, buf, n + 1)
    return buf.value.decode()


def test_bench_plan_world8_issue_sequence_and_replay(stub):
    world, D, h, P = 8, 128, 4, 65_537
    full = [torch.randn(P, generator=torch.Generator().manual_seed(500 + g)) for g in range(D)]
    shards, comms = [], []
    for r in range(world):
        rc = stub_transport(stub, r, world)
        shard, info = make_ring_shard(r, world, D, h, h, P, "cpu", ViaRccl(rc), None)
        assert info["route"]["relay"] and info["route"]["stages"] == h  # the bench's relayed, staged plan
        for i in range(shard.plan.L):
            shard.models[i] = full[shard.plan.first + i]
        shard.exchange(FakeStream(0x5000 + r))
        shards.append(shard)
        comms.append(rc.comm)
    plan = shards[0]._route_plan
    logs = [parse(read_log(stub, c)) for c in comms]

    # (1) every rank issued exactly its rank_ops per group, in order, on its stream
    for r, shard in enumerate(shards):
        routed = shard.routed()
        expect = []
        for g in range(len(plan.groups)):
            sends, recvs = plan.rank_ops(r, g)
            ops = [("send", m.dst, m.count, routed_view(routed, shard, m.src_key, m.src_off, m.count)) for m in sends]
            ops += [("recv", m.src, m.count, routed_view(routed, shard, m.dst_key, m.dst_off, m.count)) for m in recvs]
            ops = [o for o in ops if o[2] > 0]
            if ops:
                expect.append(ops)
        got = [[(op, peer, cnt, ptr) for op, peer, cnt, ptr, _ in grp] for grp in logs[r]]
        assert got == expect, f"rank {r}"
        assert all(s == 0x5000 + r for grp in logs[r] for *_, s in grp)

    # (2) + (3) pairing across ranks and the replay of every group as memory copies
    assert all(len(lg) == len(plan.groups) for lg in logs)  # every rank takes part in every group here
    for g in range(len(plan.groups)):
        for a in range(world):
            for b in range(world):
                sends = [(c, p) for op, peer, c, p, _ in logs[a][g] if op == "send" and peer == b]
                recvs = [(c, p) for op, peer, c, p, _ in logs[b][g] if op == "recv" and peer == a]
                assert [c for c, _ in sends] == [c for c, _ in recvs], (g, a, b)
                for (c, src), (_, dst) in zip(sends, recvs):
                    ctypes.memmove(dst, src, c * 4)
    for shard in shards:
        for i in shard.plan.boundary():
            g = shard.plan.first + i
            for src, j in zip(shard.sources(i), shard.plan.neighbours(g)):
                assert torch.equal(src, full[j]), (shard.plan.rank, g, j)


class RecordingLane:
    """Stands in for hostlane.HostLane in a one-process run of all ranks: records that the round
    issued its lane part (the lane's own protocol is tested in test_host_lane.py)."""

    def __init__(self):
        self.rounds = 0

    def run(self, stream=None, timing=False):
        self.rounds += 1
        return {}

    def pump(self):
        pass

    def finish(self):
        self.finished = self.rounds


def test_bench_plan_world8_with_the_host_lane(stub):
    """The bench's N = 8 plan with the host lane offered (every link alike: the planner keeps relays
    AND the lane): RCCL is handed exactly the plan's transport messages (no lane piece reaches it),
    they pair across ranks, and replaying them as copies plus the lane pieces as copies delivers
    every halo row."""
    from federated_amd.halo import RoutePlan, ring_transfers
    from federated_amd.population import RingPopulationShard, RingShardPlan
    world, D, h, P = 8, 128, 4, 65_537
    L = D // world
    plan = RoutePlan(world, ring_transfers(world, L, h, h, P), relay=True, lane=True)
    assert plan.relay and plan.lane and plan.lane_elems() > 0
    full = [torch.randn(P, generator=torch.Generator().manual_seed(900 + g)) for g in range(D)]
    shards, comms, lanes = [], [], []
    for r in range(world):
        rc = stub_transport(stub, r, world)
        shard = RingPopulationShard(RingShardPlan(r, world, L, h), P, "cpu", ViaRccl(rc), None, route=plan, rank=r)
        shard.lane = RecordingLane()
        for i in range(L):
            shard.models[i] = full[shard.plan.first + i]
        shard.exchange(FakeStream(0x6000 + r))
        shards.append(shard)
        comms.append(rc.comm)
        lanes.append(shard.lane)
    assert all(ln.rounds == 1 and ln.finished == 1 for ln in lanes)  # exchange() finishes the lane's round
    logs = [parse(read_log(stub, c)) for c in comms]
    n_lane = 0
    for r, shard in enumerate(shards):
        routed = shard.routed()
        sent = [(op, peer, cnt) for grp in logs[r] for op, peer, cnt, _, _ in grp]
        expect = []
        for g in range(len(plan.groups)):
            sends, recvs = plan.rank_ops(r, g)
            expect += [("send", m.dst, m.count) for m in sends] + [("recv", m.src, m.count) for m in recvs]
        assert sent == expect, f"rank {r}"
        n_lane += len(plan.lane_ops(r)[0])
    assert n_lane > 0
    # replay: the RCCL groups in order, then the lane pieces (they land by the last group here)
    for g in range(len(plan.groups)):
        for a in range(world):
            for b in range(world):
                sends = [(c, p) for op, peer, c, p, _ in logs[a][g] if op == "send" and peer == b]
                recvs = [(c, p) for op, peer, c, p, _ in logs[b][g] if op == "recv" and peer == a]
                assert [c for c, _ in sends] == [c for c, _ in recvs], (g, a, b)
                for (c, src), (_, dst) in zip(sends, recvs):
                    ctypes.memmove(dst, src, c * 4)
    for a in range(world):
        for m in plan.lane_ops(a)[0]:
            src = shards[a].buffer(m.src_key).reshape(-1)[m.src_off:m.src_off + m.count]
            shards[m.dst].buffer(m.dst_key).reshape(-1)[m.dst_off:m.dst_off + m.count].copy_(src)
    for shard in shards:
        for i in shard.plan.boundary():
            g = shard.plan.first + i
            for src, j in zip(shard.sources(i), shard.plan.neighbours(g)):
                assert torch.equal(src, full[j]), (shard.plan.rank, g, j)


def routed_view(routed, shard, key, off, cnt):
    buf = routed.relay[key[1]] if isinstance(key, tuple) and key[0] == "relay" else shard.buffer(key)
    return buf.reshape(-1)[off:off + cnt].data_ptr()


def test_invalid_peer_issues_nothing(stub):
    t = stub_transport(stub, 0, 2)
    a = torch.zeros(8)
    with pytest.raises(_lib.CFAError, match="bad peer"):
        t.prepare([(DeviceView(a), 2)], [])(FakeStream(1))
    assert read_log(stub, t.comm) == ""


def test_halo_exchange_and_collectives_forward_to_rccl(stub):
    t = stub_transport(stub, 1, 4)
    a, b = torch.zeros(16), torch.zeros(16)
    L = t._lib
    L.call("cfa_halo_exchange_f32", t.comm, L.ptr_table([a.data_ptr()]), L.int_array([2]), 1,
           L.ptr_table([b.data_ptr()]), L.int_array([0]), 1, 16, 7)
    L.call("cfa_allreduce_sum_f32", t.comm, a.data_ptr(), a.data_ptr(), 16, 7)
    L.call("cfa_reduce_sum_f32", t.comm, a.data_ptr(), b.data_ptr(), 16, 3, 7)
    lines = read_log(stub, t.comm).splitlines()
    assert lines == ["start", f"send 2 16 {a.data_ptr()} 7", f"recv 0 16 {b.data_ptr()} 7", "end",
                     f"allreduce 16 {a.data_ptr()} {a.data_ptr()}", f"reduce 3 16 {a.data_ptr()} {b.data_ptr()}"]
    assert np.all(a.numpy() == 0)


def test_rccl_failure_carries_rccl_text(stub):
    """An RCCL call that fails returns CFA_E_RCCL with ncclGetErrorString AND RCCL's own last
    warning (ncclGetLastError), so a bench line's headline_fallback.error says why (round-4 review).
    cfa_halo_exchange_f32 does not pre-validate peers: the stub's ncclSend refuses peer 9."""
    t = stub_transport(stub, 0, 2)
    a = torch.zeros(8)
    L = t._lib
    with pytest.raises(_lib.CFAError, match=r"ncclSend to 9: ncclInvalidArgument \[rccl: stub: peer refused\]"):
        L.call("cfa_halo_exchange_f32", t.comm, L.ptr_table([a.data_ptr()]), L.int_array([9]), 1,
               L.ptr_table([]), L.int_array([]), 0, 8, 7)
