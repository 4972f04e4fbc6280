"""In-process loopback transport: N shards of a sharded population on ONE GPU, one host thread
per shard, their halo exchanged by device-to-device ``hipMemcpyAsync``.

The multi-GPU path (SURVEY §8 e) shards the simulated population one block per rank and moves the
cross-shard neighbour buckets with grouped RCCL send/recv (``cfa_p2p_group_f32``). A one-GPU box
cannot open an RCCL communicator of more than one rank ("Duplicate GPU"), so the sharded BASELINE
configs -- C4, CIFAR-100 VGG-1 over 4 shards (TF2 ``...FL_threads_CIFAR100.py:160-170,442-450``),
and C5, the radar ring over 8 shards (``consensus_v4.py:133-137``) -- are exercised here with
every shard's HIP kernels on the same card and this transport in place of RCCL. It obeys the
semantics the shards rely on from ``cfa_p2p_group_f32``:

- one ``exchange(sends, recvs, stream)`` call is one group: messages between one rank pair pair
  up in issue order (FIFO per ordered pair); zero-length messages are skipped on both sides;
- the receive lands on the receiver's ``stream`` after the sender's ``stream`` has reached the
  group (an event recorded at issue), and the sender's ``stream`` continues only after the copy
  has completed (it waits on an event the receiver records after the copy): a send buffer is
  never overwritten while a peer is still reading it, as with a completed NCCL group;
- a group waits (on the host) for its peers' matching calls, so a mismatched schedule fails with
  a timeout that names the rank pair instead of hanging, and a rank that fails ends every other
  rank's wait with its message.

Host (CPU) buffers are accepted too, copied synchronously: the CPU suite runs the same schedules
(e.g. the routed, relayed halo plan at world 8) through this transport without a GPU.

``allreduce_sum`` / ``reduce_sum`` sum the ranks' buffers in rank order (deterministic).

This is test and rehearsal plumbing for the sharded path; the product transport is
``dist.RcclTransport``.
"""
from __future__ import annotations

import collections
import contextlib
import threading
from typing import Callable, List, Optional, Sequence

import torch

from federated_amd import _lib

Transfer = tuple  # (contiguous fp32 CUDA tensor, peer rank)


class LoopbackError(RuntimeError):
    pass


class _Msg:
    __slots__ = ("buf", "ready", "done", "done_ev", "error")

    def __init__(self, buf: torch.Tensor, ready):
        self.buf, self.ready = buf, ready
        self.done = False
        self.done_ev = None
        self.error: Optional[str] = None


def _record(stream):
    """An event at the current end of ``stream`` (None for host buffers: copies are synchronous)."""
    if stream is None:
        return None
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


class LoopbackHub:
    """Shared state of the ``world`` in-process ranks: FIFO message queues per ordered rank pair
    and the collective rendezvous. Every wait is bounded by ``timeout`` and ends early, with the
    failing rank's message, when another rank has failed."""

    def __init__(self, world: int, timeout: float = 120.0):
        if world < 1:
            raise ValueError("world must be >= 1")
        self.world, self.timeout = int(world), float(timeout)
        self.cv = threading.Condition()
        self.queues = collections.defaultdict(collections.deque)  # (src, dst) -> deque[_Msg]
        self._coll_gen = 0
        self._coll_posts: dict = {}
        self._coll_done: dict = {}
        self.failed: Optional[str] = None
        self.failed_rank: Optional[int] = None  # the rank whose failure came first (the cause)
        self.groups = [0] * self.world  # exchange calls per rank
        self.messages = [0] * self.world  # non-empty messages received per rank

    def transport(self, rank: int) -> "LoopbackTransport":
        return LoopbackTransport(self, rank)

    def fail(self, why: str, rank: Optional[int] = None) -> None:
        with self.cv:
            if self.failed is None:
                self.failed, self.failed_rank = why, rank
            self.cv.notify_all()

    def _wait(self, pred: Callable[[], bool], what: str) -> None:
        """Caller holds cv."""
        if not self.cv.wait_for(lambda: pred() or self.failed is not None, timeout=self.timeout):
            raise LoopbackError(f"loopback: timed out after {self.timeout:.0f} s waiting for {what}")
        if not pred():
            raise LoopbackError(f"loopback: gave up waiting for {what}: {self.failed}")


class LoopbackTransport:
    name = "loopback"
    host_staged = False

    def __init__(self, hub: LoopbackHub, rank: int):
        if not 0 <= rank < hub.world:
            raise ValueError(f"rank {rank} outside world {hub.world}")
        self.hub, self.rank, self.world = hub, int(rank), hub.world

    @staticmethod
    def _check(buf: torch.Tensor) -> None:
        if not (buf.dtype == torch.float32 and buf.is_contiguous()):
            raise TypeError("exchange buffers must be contiguous fp32 tensors")

    @staticmethod
    def _stream(buf: torch.Tensor, stream):
        if not buf.is_cuda:
            return None
        return stream if stream is not None else torch.cuda.current_stream(buf.device)

    @staticmethod
    def _copy(dst: torch.Tensor, src: torch.Tensor, stream) -> None:
        if stream is None:
            dst.copy_(src)
            return
        _lib.call("cfa_memcpy_async", dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size(),
                  int(stream.cuda_stream))

    def exchange(self, sends: Sequence[Transfer], recvs: Sequence[Transfer], stream=None) -> None:
        hub, me = self.hub, self.rank
        bufs = list(sends) + list(recvs)
        for b, p in bufs:
            self._check(b)
            if not 0 <= p < self.world:
                raise ValueError(f"peer {p} outside world {self.world}")
        if len({b.is_cuda for b, _ in bufs}) > 1:
            raise TypeError("a group's buffers must all be device or all host tensors")
        s = self._stream(bufs[0][0], stream) if bufs else None
        try:
            self._group(sends, recvs, s)
        except BaseException as exc:
            hub.fail(f"rank {me}: {exc}", me)
            raise

    def _group(self, sends, recvs, s) -> None:
        hub, me = self.hub, self.rank
        posted: List[_Msg] = []
        with hub.cv:
            hub.groups[me] += 1
            for b, p in sends:
                if b.numel() == 0:
                    continue
                m = _Msg(b, _record(s))
                hub.queues[(me, p)].append(m)
                posted.append(m)
            hub.cv.notify_all()
        for b, p in recvs:
            if b.numel() == 0:
                continue
            with hub.cv:
                q = hub.queues[(p, me)]
                hub._wait(lambda: len(q) > 0, f"a message from rank {p} to rank {me}")
                m = q.popleft()
            if m.buf.numel() != b.numel():
                with hub.cv:
                    m.error = f"rank {p} sent {m.buf.numel()} floats, rank {me} receives {b.numel()}"
                    m.done = True
                    hub.cv.notify_all()
                raise LoopbackError("loopback: " + m.error)
            if s is not None:
                s.wait_event(m.ready)
            self._copy(b, m.buf, s)
            ev = _record(s)
            with hub.cv:
                m.done_ev, m.done = ev, True
                hub.messages[me] += 1
                hub.cv.notify_all()
        for m in posted:
            with hub.cv:
                hub._wait(lambda: m.done, f"rank {me}'s send of {m.buf.numel()} floats to be received")
            if m.error:
                raise LoopbackError("loopback: " + m.error)
            if s is not None:
                s.wait_event(m.done_ev)

    def _rendezvous(self, buf: torch.Tensor, stream) -> tuple:
        """All ranks post (buffer, ready event); returns (generation, posts in rank order)."""
        hub = self.hub
        ev = _record(stream)
        with hub.cv:
            gen = hub._coll_gen
            posts = hub._coll_posts.setdefault(gen, {})
            posts[self.rank] = (buf, ev)
            if len(posts) == self.world:
                hub._coll_gen += 1
                hub.cv.notify_all()
            else:
                hub._wait(lambda: len(posts) == self.world, f"collective {gen} (rank {self.rank})")
        return gen, [posts[r] for r in range(self.world)]

    def _finish(self, gen: int, stream) -> None:
        """Second barrier: no rank overwrites its buffer before every rank has read all of them."""
        hub = self.hub
        ev = _record(stream)
        with hub.cv:
            done = hub._coll_done.setdefault(gen, {})
            done[self.rank] = ev
            if len(done) == self.world:
                # every rank has read every post: drop the generation's entries (the waiting ranks
                # hold `done` themselves), so a long run keeps no buffers alive
                hub._coll_posts.pop(gen, None)
                hub._coll_done.pop(gen, None)
                hub.cv.notify_all()
            else:
                hub._wait(lambda: len(done) == self.world, f"collective {gen} completion (rank {self.rank})")
        if stream is not None:
            for r in range(self.world):
                stream.wait_event(done[r])

    def _sum(self, buf: torch.Tensor, stream, write: bool) -> None:
        self._check(buf)
        s = self._stream(buf, stream)
        try:
            gen, posts = self._rendezvous(buf, s)
            if any(b.numel() != buf.numel() or b.is_cuda != buf.is_cuda for b, _ in posts):
                raise LoopbackError("loopback: collective buffers differ across ranks")
            if s is not None:
                for _, ev in posts:
                    s.wait_event(ev)
            with torch.cuda.stream(s) if s is not None else contextlib.nullcontext():
                acc = posts[0][0].clone()
                for b, _ in posts[1:]:
                    acc.add_(b)
            self._finish(gen, s)
            if write:
                with torch.cuda.stream(s) if s is not None else contextlib.nullcontext():
                    buf.copy_(acc)
        except BaseException as exc:
            self.hub.fail(f"rank {self.rank}: {exc}", self.rank)
            raise

    def allreduce_sum(self, buf: torch.Tensor, stream=None) -> None:
        self._sum(buf, stream, True)

    def reduce_sum(self, buf: torch.Tensor, root: int, stream=None) -> None:
        self._sum(buf, stream, self.rank == int(root))

    def close(self) -> None:
        pass


def run_ranks(world: int, fn: Callable[[int, LoopbackTransport], object], timeout: float = 300.0,
              hub: Optional[LoopbackHub] = None) -> list:
    """Run ``fn(rank, transport)`` for every rank, one host thread each, on a shared hub; returns
    the results in rank order, or re-raises the exception of the rank that failed first."""
    hub = hub or LoopbackHub(world)
    results: list = [None] * world
    errors: list = [None] * world
    device = torch.cuda.current_device() if torch.cuda.is_available() else None

    def body(r):
        try:
            if device is not None:
                torch.cuda.set_device(device)
            results[r] = fn(r, hub.transport(r))
        except BaseException as exc:  # noqa: BLE001 - re-raised on the caller's thread
            errors[r] = exc
            hub.fail(f"rank {r}: {type(exc).__name__}: {exc}", r)

    threads = [threading.Thread(target=body, args=(r,), name=f"loopback-rank{r}", daemon=True) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout)
        if t.is_alive():
            raise LoopbackError(f"loopback: {t.name} still running after {timeout:.0f} s")
    first = hub.failed_rank
    if first is not None and errors[first] is not None:
        raise errors[first]  # the cause, not another rank's "gave up waiting"
    for e in errors:
        if e is not None:
            raise e
    return results
