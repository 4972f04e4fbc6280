"""Host lane: part of a round's halo travels over PCIe through shared pinned host memory, beside xGMI.

Two GPUs of an MI355X node share exactly one xGMI link, so with the population sharded in device
blocks over N = 2 GPUs the whole ring halo (800 MB per rank per round at the bench's shape) rides
one link direction, and at N = 4 two; the mixes of a round take half that long.
The only other path between two GPUs is each GPU's PCIe Gen5 x16 link to host memory (63 GB/s
per direction spec; 55 GB/s D2H and H2D measured, 50 + 55 GB/s with both at once in 32 MB
copies, ``profiles/r05_host_lane_chunk_sweep.jsonl``). The reference has no such path to mirror: its devices
exchange models as files (TF1 ``cfa.py:119-130``).

A lane piece (``halo.RoutePlan`` with ``lane=True``) goes:

    sender: D2H copy of the piece's chunk into the pair's shared segment  -> raise READY to its number
    receiver: wait (on the GPU) until READY reaches that number  -> H2D copy into the halo row

Both ends are stream-ordered on the GPU: the sender's ``cfa_stream_signal`` (a one-lane
system-scope release store into the pinned segment) follows its copy on the lane's out stream; the
receiver's ``cfa_stream_wait_word`` (a one-lane kernel polling that word, with a timeout that
every wave reaches) precedes its copy on the lane's in stream. The host only enqueues. Segments:
one per (sender, receiver) pair that carries lane pieces, a POSIX shared-memory file created by the
sender, mapped and pinned (``cfa_host_register``) by both, unlinked as soon as both hold it; two
round parities of data, so the sender of round r waits only for the receiver's ACK of round
r - 2. Chunks of ``chunk_elems`` keep D2H and H2D pipelined (a whole-row copy would serialise
them).

The same protocol runs on CPU tensors (gloo tests): copies are ``torch`` copies between the
segment and the buffers and the words are read and written by the host, so the cross-process
protocol (layout, sequence numbers, parities, back-pressure) is tested without a GPU.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import time
from typing import Callable, Dict, Hashable, List, Optional, Sequence, Tuple

import torch

from .halo import ALIGN, Message

FLAG_BYTES = 4096
READY, ACK = 0, 16            # u32 word indices in a segment's flag page (64 bytes apart)
# 32 MiB fp32 copies: with D2H and H2D at once, 49.6 + 54.7 GB/s against 47.1 + 53.5 at 16 MiB and
# 39.1 + 40.6 at 2 MiB; 64 MiB adds < 1%, 100 MiB halves the H2D (r05_host_lane_chunk_sweep.jsonl)
DEFAULT_CHUNK_ELEMS = 8 << 20
RAMP = 3  # a pair's round starts with chunks of 1/8, 1/4, 1/2 of that: the H2D starts after 4 MiB
DEFAULT_TIMEOUT_S = 60.0
SHM_DIR = "/dev/shm"


def lane_layout(msgs: Sequence[Message], align: int = ALIGN) -> Tuple[List[int], int]:
    """Element offsets of ``msgs`` (one sender -> receiver pair, global message order) packed in
    one parity of the pair's segment, each ``align``-aligned; and the parity's length. Sender and
    receiver compute it from the same plan, so they agree without talking."""
    offs, n = [], 0
    for m in msgs:
        offs.append(n)
        n += -(-m.count // align) * align
    return offs, n


def first_chunk_elems(chunk_elems: int, ramp: int = RAMP) -> int:
    """Elements of a pair's first chunk in a round (what the receiver waits for before its first
    H2D can start: the lane pipeline's fill)."""
    return max(ALIGN, (int(chunk_elems) >> ramp) // ALIGN * ALIGN)


def lane_chunks(msgs: Sequence[Message], offs: Sequence[int], chunk_elems: int,
                ramp: int = RAMP) -> List[Tuple[int, int, int, int]]:
    """The pair's copies of one round in order: (message index, element offset within the
    message, elements, segment offset). Messages are cut in pieces of ``chunk_elems``, except the
    round's first ``ramp`` pieces, which grow from chunk_elems / 2**ramp by doubling (aligned), so
    the receiver's first H2D waits for a small D2H only."""
    out, k = [], 0
    for i, m in enumerate(msgs):
        lo = 0
        while lo < m.count:
            size = chunk_elems if k >= ramp else first_chunk_elems(chunk_elems, ramp - k)
            n = min(size, m.count - lo)
            out.append((i, lo, n, offs[i] + lo))
            lo += n
            k += 1
    return out


def segment_path(token: str, src: int, dst: int) -> str:
    return os.path.join(SHM_DIR, f"cfa_lane_{token}_{src}_{dst}")


class _Segment:
    """One direction's shared segment: [2 parities x ``elems`` fp32] then a flag page."""

    def __init__(self, path: str, elems: int, create: bool):
        self.path, self.elems = path, int(elems)
        self.data_bytes = 2 * self.elems * 4
        self.size = self.data_bytes + FLAG_BYTES
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                # reserve the pages now: a full /dev/shm fails here (ENOSPC, reported through the
                # open's agreement) instead of a SIGBUS at the first copy into a sparse file
                os.posix_fallocate(fd, 0, self.size)
            self.mm = mmap.mmap(fd, self.size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self._anchor = ctypes.c_char.from_buffer(self.mm)  # exports of the mapping: dropped in close()
        self.base = ctypes.addressof(self._anchor)
        self.words = (ctypes.c_uint32 * (FLAG_BYTES // 4)).from_buffer(self.mm, self.data_bytes)
        self.data = torch.frombuffer(self.mm, dtype=torch.float32, count=2 * self.elems) if self.elems else None
        self.dev_base = None
        self._lib = None

    def register(self, lib) -> None:
        from . import _lib
        _lib.check("cfa_host_register", lib.cfa_host_register(ctypes.c_void_p(self.base), self.size))
        self._lib = lib
        dp = ctypes.c_void_p()
        _lib.check("cfa_host_device_pointer", lib.cfa_host_device_pointer(ctypes.c_void_p(self.base), ctypes.byref(dp)))
        self.dev_base = dp.value

    def host_ptr(self, parity: int, off: int) -> int:
        return self.base + (parity * self.elems + off) * 4

    def word_dev(self, i: int) -> int:
        return self.dev_base + self.data_bytes + 4 * i

    def read(self, i: int) -> int:
        return int(self.words[i])

    def close(self) -> None:
        """Unpin, drop this object's exports of the mapping and unmap it (the pages go once the
        peer has unmapped too; the name was unlinked at open)."""
        if self._lib is not None:
            self._lib.cfa_host_unregister(ctypes.c_void_p(self.base))
            self._lib = None
        if self.mm is not None:
            self.data = self.words = self._anchor = None
            try:
                self.mm.close()
            except BufferError:  # a caller still holds a view of the segment: it stays mapped
                pass
            self.mm = None


def _reached(word: int, value: int) -> bool:
    """Sequence order of 32-bit counters (what the wait kernel tests: (int)(word - value) >= 0)."""
    return ((word - value) & 0xFFFFFFFF) < 0x80000000


class HostLane:
    """The host-lane messages of one rank, bound to its buffers and the pair segments.

    Build with ``HostLane.open`` (collective: every rank of the plan calls it). ``run(stream)``
    issues one round's lane copies after ``stream``'s earlier work and returns
    {group index: event after the H2D copies of that group's pieces} (GPU) or {} (CPU, where
    ``run`` returns once every piece has landed)."""

    def __init__(self, rank: int, sends: Sequence[Message], recvs: Sequence[Message],
                 buffers: Callable[[Hashable], torch.Tensor], device, token: str,
                 chunk_elems: int = DEFAULT_CHUNK_ELEMS, timeout_s: float = DEFAULT_TIMEOUT_S):
        self.rank, self.token = int(rank), str(token)
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.chunk_elems = max(ALIGN, int(chunk_elems) // ALIGN * ALIGN)
        self.timeout_s = float(timeout_s)
        self.round = 0
        self.out_msgs: Dict[int, List[Message]] = {}
        self.in_msgs: Dict[int, List[Message]] = {}
        for m in sends:
            if m.src != self.rank or not m.lane:
                raise ValueError(f"rank {rank}: {m} is not one of its lane sends")
            self.out_msgs.setdefault(m.dst, []).append(m)
        for m in recvs:
            if m.dst != self.rank or not m.lane:
                raise ValueError(f"rank {rank}: {m} is not one of its lane receives")
            self.in_msgs.setdefault(m.src, []).append(m)

        def view(key, off, cnt):
            return buffers(key).reshape(-1)[off:off + cnt]

        self._out_views = {d: [view(m.src_key, m.src_off, m.count) for m in ms] for d, ms in self.out_msgs.items()}
        self._in_views = {s: [view(m.dst_key, m.dst_off, m.count) for m in ms] for s, ms in self.in_msgs.items()}
        for views in list(self._out_views.values()) + list(self._in_views.values()):
            for v in views:
                if v.dtype != torch.float32 or v.device != self.device:
                    raise ValueError(f"host lane buffers must be fp32 on {self.device}")
        self.out_seg: Dict[int, _Segment] = {}
        self.in_seg: Dict[int, _Segment] = {}
        self._lib = None
        self._status = None
        self.last_timing = None

    # -- setup --------------------------------------------------------------------------------
    def _layout(self, msgs):
        offs, n = lane_layout(msgs)
        return offs, n, lane_chunks(msgs, offs, self.chunk_elems)

    def create_segments(self) -> None:
        for dst, ms in sorted(self.out_msgs.items()):
            _, n, _ = self._layout(ms)
            self.out_seg[dst] = _Segment(segment_path(self.token, self.rank, dst), n, create=True)

    def open_segments(self) -> None:
        for src, ms in sorted(self.in_msgs.items()):
            _, n, _ = self._layout(ms)
            self.in_seg[src] = _Segment(segment_path(self.token, src, self.rank), n, create=False)
        if self.gpu:
            from . import _lib
            self._lib = _lib.load()
            for seg in list(self.out_seg.values()) + list(self.in_seg.values()):
                seg.register(self._lib)
            # [out-stream timeout, in-stream timeout]: written by the wait kernels that time out
            self._status = torch.zeros(2, dtype=torch.int32, pin_memory=True)
            dp = ctypes.c_void_p()
            _lib.check("cfa_host_device_pointer",
                       self._lib.cfa_host_device_pointer(ctypes.c_void_p(self._status.data_ptr()), ctypes.byref(dp)))
            self._status_dev = dp.value
            self.out_stream = torch.cuda.Stream(self.device)
            self.in_stream = torch.cuda.Stream(self.device)
        self._plan_round()

    def unlink(self) -> None:
        """Remove the names of the segments this rank created (both ends hold their mappings)."""
        for seg in self.out_seg.values():
            try:
                os.unlink(seg.path)
            except FileNotFoundError:
                pass

    @classmethod
    def open(cls, rank: int, sends, recvs, buffers, device, token: str, agree: Callable[[bool], bool],
             **kw) -> "HostLane":
        """Collective over the ranks of the plan: create this rank's outgoing segments, agree, map
        and pin the incoming ones, agree, unlink the names. ``agree(ok)`` is the control plane's
        all-ranks AND (it doubles as the barrier): a failure on any rank raises on every rank, so
        none is left waiting for a peer that gave up."""
        lane = cls(rank, sends, recvs, buffers, device, token, **kw)
        err = None
        try:
            lane.create_segments()
        except Exception as exc:  # reported on every rank below
            err = f"{type(exc).__name__}: {exc}"
        if not agree(err is None):
            lane.unlink()
            raise RuntimeError(f"host lane: creating the segments failed ({err or 'on another rank'})")
        try:
            lane.open_segments()
        except Exception as exc:
            err = f"{type(exc).__name__}: {exc}"
        ok = agree(err is None)
        lane.unlink()
        if not ok:
            lane.close()
            raise RuntimeError(f"host lane: mapping the segments failed ({err or 'on another rank'})")
        return lane

    def _plan_round(self) -> None:
        """Per pair: the copies of a round in group order (the sender interleaves its peers group
        by group, so every receiver's early stages leave first)."""
        self._out_plan = []  # (group, dst, chunk number, segment offset, source slice)
        per_dst = {}
        for dst, ms in self.out_msgs.items():
            offs, n, chunks = self._layout(ms)
            per_dst[dst] = [(ms[i].group, dst, k, so, self._out_views[dst][i][lo:lo + c])
                            for k, (i, lo, c, so) in enumerate(chunks)]
        self._out_n = {d: len(c) for d, c in per_dst.items()}
        self._out_plan = sorted((x for c in per_dst.values() for x in c), key=lambda x: (x[0], x[2], x[1]))
        self._in_plan = []
        self._in_n = {}
        for src, ms in self.in_msgs.items():
            offs, n, chunks = self._layout(ms)
            self._in_n[src] = len(chunks)
            self._in_plan += [(ms[i].group, src, k, so, self._in_views[src][i][lo:lo + c])
                              for k, (i, lo, c, so) in enumerate(chunks)]
        self._in_plan.sort(key=lambda x: (x[0], x[2], x[1]))
        self._groups = sorted({x[0] for x in self._in_plan})

    # -- one round -------------------------------------------------------------------------------
    @property
    def elems_out(self) -> int:
        return sum(m.count for ms in self.out_msgs.values() for m in ms)

    @property
    def elems_in(self) -> int:
        return sum(m.count for ms in self.in_msgs.values() for m in ms)

    def check(self) -> None:
        """Raise if a wait of an earlier round timed out (GPU: the wait kernels' status words)."""
        if self._status is not None:
            st = self._status.tolist()
            if any(st):
                raise RuntimeError(f"host lane rank {self.rank}: a wait timed out after {self.timeout_s:.0f} s "
                                   f"(out-stream status {st[0]}, in-stream status {st[1]}): the peer's "
                                   "copies never landed")

    def run(self, stream=None, timing: bool = False) -> Dict[int, object]:
        """One round's lane copies; see the class docstring. ``timing`` records HIP events at the
        start and end of each stream's work (``last_timing``: out / in milliseconds, per-group in
        arrival ms), for the bench's decomposition."""
        self.check()
        r = self.round
        self.round += 1
        if not self.gpu:
            self._run_cpu(r)
            return {}
        return self._run_gpu(r, stream, timing)

    def _run_gpu(self, r: int, stream, timing: bool) -> Dict[int, object]:
        from . import _lib
        lib = self._lib
        par = r & 1
        tmo = int(self.timeout_s * 1e6)
        os_, is_ = self.out_stream, self.in_stream
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        os_.wait_stream(st)  # the rows are final before they leave
        is_.wait_stream(st)  # the halo rows are no longer read when they are overwritten
        osh, ish = ctypes.c_void_p(os_.cuda_stream), ctypes.c_void_p(is_.cuda_stream)
        ev = None
        if timing:
            ev = {"o0": torch.cuda.Event(enable_timing=True), "o1": torch.cuda.Event(enable_timing=True),
                  "i0": torch.cuda.Event(enable_timing=True), "i1": torch.cuda.Event(enable_timing=True)}
            ev["o0"].record(os_)
            ev["i0"].record(is_)
        if r >= 2:  # the receiver has drained round r - 2 from this parity
            for dst, seg in self.out_seg.items():
                _lib.check("cfa_stream_wait_word", lib.cfa_stream_wait_word(
                    ctypes.c_void_p(seg.word_dev(ACK)), (r - 1) & 0xFFFFFFFF, tmo, ctypes.c_void_p(self._status_dev),
                    osh))
        for g, dst, k, so, src in self._out_plan:
            seg = self.out_seg[dst]
            _lib.check("cfa_memcpy_async", lib.cfa_memcpy_async(ctypes.c_void_p(seg.host_ptr(par, so)),
                                                               ctypes.c_void_p(src.data_ptr()), src.numel() * 4, osh))
            seq = (r * self._out_n[dst] + k + 1) & 0xFFFFFFFF
            _lib.check("cfa_stream_signal", lib.cfa_stream_signal(ctypes.c_void_p(seg.word_dev(READY)), seq, osh))
        events = {}
        last = {}
        for i, (g, src_rank, k, so, dst) in enumerate(self._in_plan):
            last[g] = i
        for i, (g, src_rank, k, so, dst) in enumerate(self._in_plan):
            seg = self.in_seg[src_rank]
            seq = (r * self._in_n[src_rank] + k + 1) & 0xFFFFFFFF
            _lib.check("cfa_stream_wait_word", lib.cfa_stream_wait_word(
                ctypes.c_void_p(seg.word_dev(READY)), seq, tmo, ctypes.c_void_p(self._status_dev + 4), ish))
            if timing and i == 0:  # the first chunk has landed in host memory: the pipeline is full
                ev["i_first"] = torch.cuda.Event(enable_timing=True)
                ev["i_first"].record(is_)
            _lib.check("cfa_memcpy_async", lib.cfa_memcpy_async(ctypes.c_void_p(dst.data_ptr()),
                                                               ctypes.c_void_p(seg.host_ptr(par, so)), dst.numel() * 4,
                                                               ish))
            if last[g] == i:
                e = torch.cuda.Event(enable_timing=timing)
                e.record(is_)
                events[g] = e
        for src_rank, seg in self.in_seg.items():
            _lib.check("cfa_stream_signal", lib.cfa_stream_signal(ctypes.c_void_p(seg.word_dev(ACK)),
                                                                  (r + 1) & 0xFFFFFFFF, ish))
        if timing:
            ev["o1"].record(os_)
            ev["i1"].record(is_)
            ev["groups"] = events
        self.last_timing = ev
        return events

    def timing_ms(self) -> Optional[dict]:
        """After the stream has been synchronised: the last timed round's out-stream and
        in-stream milliseconds, the in-stream's steady part (from the first chunk's arrival in
        host memory to its end: every H2D, none of the sender's start-up or first D2H) and each
        group's arrival (ms from the in-stream's start)."""
        ev = self.last_timing
        if not ev:
            return None
        out = {"out_ms": ev["o0"].elapsed_time(ev["o1"]), "in_ms": ev["i0"].elapsed_time(ev["i1"]),
               "group_arrival_ms": {g: ev["i0"].elapsed_time(e) for g, e in ev["groups"].items()}}
        if "i_first" in ev:
            out["in_steady_ms"] = ev["i_first"].elapsed_time(ev["i1"])
        return out

    def wait_streams(self, stream) -> None:
        """Make ``stream`` wait for this round's lane work (both directions)."""
        if self.gpu:
            stream.wait_stream(self.out_stream)
            stream.wait_stream(self.in_stream)

    def _spin(self, seg: _Segment, word: int, value: int, what: str) -> None:
        t_end = time.monotonic() + self.timeout_s
        n = 0
        while not _reached(seg.read(word), value):
            n += 1
            if n > 64:
                time.sleep(50e-6)
            if time.monotonic() > t_end:
                raise RuntimeError(f"host lane rank {self.rank}: timed out after {self.timeout_s:.0f} s waiting for "
                                   f"{what} (word {seg.read(word)}, want {value})")

    def _run_cpu(self, r: int) -> None:
        par = r & 1
        if r >= 2:
            for dst, seg in self.out_seg.items():
                self._spin(seg, ACK, (r - 1) & 0xFFFFFFFF, f"rank {dst}'s ack of round {r - 2}")
        for g, dst, k, so, src in self._out_plan:
            seg = self.out_seg[dst]
            n = src.numel()
            seg.data[par * seg.elems + so: par * seg.elems + so + n].copy_(src)
            seg.words[READY] = (r * self._out_n[dst] + k + 1) & 0xFFFFFFFF
        for g, src_rank, k, so, dst in self._in_plan:
            seg = self.in_seg[src_rank]
            seq = (r * self._in_n[src_rank] + k + 1) & 0xFFFFFFFF
            self._spin(seg, READY, seq, f"chunk {k} of round {r} from rank {src_rank}")
            n = dst.numel()
            dst.copy_(seg.data[par * seg.elems + so: par * seg.elems + so + n])
        for src_rank, seg in self.in_seg.items():
            seg.words[ACK] = (r + 1) & 0xFFFFFFFF

    def close(self) -> None:
        """Drain the lane's streams, then unpin and drop the segments."""
        if self.gpu and hasattr(self, "out_stream"):
            self.out_stream.synchronize()
            self.in_stream.synchronize()
        for seg in list(self.out_seg.values()) + list(self.in_seg.values()):
            seg.close()
        self.out_seg, self.in_seg = {}, {}

    def summary(self) -> dict:
        return {"token": self.token, "chunk_MB": round(self.chunk_elems * 4 / 2**20, 2),
                "out_MB": round(self.elems_out * 4 / 1e6, 2), "in_MB": round(self.elems_in * 4 / 1e6, 2),
                "peers_out": sorted(self.out_msgs), "peers_in": sorted(self.in_msgs)}


def new_token() -> str:
    """A job-unique segment-name token (rank 0 draws it; the caller broadcasts it)."""
    return f"{os.getpid()}_{int.from_bytes(os.urandom(4), 'little'):08x}"
