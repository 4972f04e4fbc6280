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
    receiver: its HOST sees READY reach that number  -> enqueues the H2D copy into the halo row

The sender's side is stream-ordered: ``cfa_stream_signal`` (a one-lane system-scope release store
into the pinned segment) follows each D2H copy on the lane's out stream. The receiver's waits are
on the host, never on a GPU queue (round 6): a native pump thread of the lane's own
(``cfa_lane_pump_*``, csrc/cfa_lane.cpp) polls each chunk's word (acquire loads) and only then
enqueues the chunk's H2D on the lane's in stream, then the group's event, and at the round's end
the ACKs. A wait parked on the GPU held every stream sharing its hardware queue (HIP maps a
process's streams onto ``GPU_MAX_HW_QUEUES``, 4 on this pool), the compute stream included; a
host wait holds nothing, and on its own thread it does not hold the round's thread either (which
may be inside a blocking transport call). ``run`` enqueues the D2H side and submits the receive
side to the pump; before each boundary set a gate's ``wait(stream)`` blocks until the pump has
enqueued that set's chunks and then makes the stream wait on their event; ``finish`` waits for the
whole round. A wait that times out fails the round whose chunk it was (``LaneTimeout``), and the
lane refuses every later round.

Segments: one per (sender, receiver) pair that carries lane pieces, a POSIX shared-memory file
created by the sender, its pages reserved with the policy "prefer the RECEIVER's NUMA node"
(``numa.py``; the receiver's H2D reads local memory), mapped and pinned (``cfa_host_register``) by
both, unlinked as soon as both hold it; two round parities of data, so the sender of round r waits
(on the host) only for the receiver's ACK of round r - 2. Chunks of ``chunk_elems`` keep D2H and
H2D pipelined (a whole-row copy would serialise them).

The same protocol runs on CPU tensors (gloo tests): the send side's copies are ``torch`` copies
and its words host stores, and the receive side runs on the same native pump in host mode
(memcpy, host stores), so the cross-process protocol (layout, sequence numbers, parities,
back-pressure, timeouts) is tested without a GPU.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import weakref
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


class LaneTimeout(RuntimeError):
    """A host-lane wait gave up: the peer's copy (or ACK) never arrived."""


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

    def __init__(self, path: str, elems: int, create: bool, numa_node: Optional[int] = None):
        self.path, self.elems = path, int(elems)
        self.data_bytes = 2 * self.elems * 4
        self.size = self.data_bytes + FLAG_BYTES
        self.numa_wanted = numa_node if create else None
        self.numa_note = None
        flags = os.O_RDWR | (os.O_CREAT | os.O_EXCL if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create:
                # reserve the pages now, preferring the receiver's NUMA node: a full /dev/shm fails
                # here (ENOSPC, reported through the open's agreement) instead of a SIGBUS at the
                # first copy into a sparse file
                from . import numa
                with numa.preferred(numa_node) as why:
                    self.numa_note = why
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

    def placed_nodes(self) -> List[Optional[int]]:
        """NUMA node of the segment's first, middle and last data page (None: not known)."""
        from . import numa
        if not self.data_bytes:
            return []
        return [numa.node_of(self.base + off) for off in
                sorted({0, self.data_bytes // 2 // 4096 * 4096, (self.data_bytes - 1) // 4096 * 4096})]

    def register(self, lib) -> None:
        from . import _lib
        _lib.check("cfa_host_register", lib.cfa_host_register(ctypes.c_void_p(self.base), self.size))
        self._lib = lib
        dp = ctypes.c_void_p()
        _lib.check("cfa_host_device_pointer", lib.cfa_host_device_pointer(ctypes.c_void_p(self.base), ctypes.byref(dp)))
        self.dev_base = dp.value

    def host_ptr(self, parity: int, off: int) -> int:
        return self.base + (parity * self.elems + off) * 4

    def word_host(self, i: int) -> int:
        return self.base + self.data_bytes + 4 * i

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
    """Sequence order of 32-bit counters (what cfa_host_wait_word tests: (int)(word - value) >= 0)."""
    return ((word - value) & 0xFFFFFFFF) < 0x80000000


class _Round:
    """One round's state while the pump works through it."""

    def __init__(self, r: int, timing: bool):
        self.r, self.timing = r, timing
        self.ops = None        # the pump's operation array (kept alive for the round)
        self.events: Dict[int, object] = {}  # group -> event after its H2D copies (GPU)
        self.ev: Dict[str, object] = {}      # timing events
        self.done = False


class LaneGate:
    """What ``HostLane.run`` hands out per group: ``wait(stream)`` blocks on the host (GIL
    released) until the lane's pump thread has enqueued the group's lane pieces (and every
    earlier group's), then makes ``stream`` wait on the event after their copies; it is what
    ``torch.cuda.Stream.wait_event`` calls, so a gate stands where an event would."""

    def __init__(self, lane: "HostLane", rnd: _Round, group: int):
        self.lane, self.rnd, self.group = lane, rnd, group

    def wait(self, stream=None) -> None:
        ev = self.lane.advance(self.group, self.rnd)
        if ev is not None:
            ev.wait(stream)


class HostLane:
    """The host-lane messages of one rank, bound to its buffers and the pair segments.

    Build with ``HostLane.open`` (collective: every rank of the plan calls it). ``run(stream)``
    starts one round after ``stream``'s earlier work and returns {group index: LaneGate}; the
    lane's pump thread enqueues the receiving side as its chunks arrive, and a gate's ``wait`` or
    ``finish()`` blocks until it has (see the module docstring). On CPU tensors the pump copies
    with memcpy (host mode)."""

    def __init__(self, rank: int, sends: Sequence[Message], recvs: Sequence[Message],
                 buffers: Callable[[Hashable], torch.Tensor], device, token: str,
                 chunk_elems: int = DEFAULT_CHUNK_ELEMS, timeout_s: float = DEFAULT_TIMEOUT_S,
                 numa_nodes: Optional[Sequence[Optional[int]]] = None, segment_elems: int = 0):
        """``numa_nodes[r]``: the NUMA node of rank r's GPU (None or absent: no placement); the
        segment a rank sends to r prefers r's node. ``segment_elems``: reserve at least this many
        elements per parity of every segment (the lane probe reserves what the headline's plan
        may need, so it fails where the headline would); both ends must pass the same value."""
        self.rank, self.token = int(rank), str(token)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:  # "cuda" means the current GPU
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.gpu = self.device.type == "cuda"
        self.chunk_elems = max(ALIGN, int(chunk_elems) // ALIGN * ALIGN)
        self.timeout_s = float(timeout_s)
        self.numa_nodes = list(numa_nodes) if numa_nodes is not None else None
        self.segment_elems = max(0, int(segment_elems))
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
        self._pump = None
        self._cur: Optional[_Round] = None
        self._last_round: Optional[_Round] = None
        self._error: Optional[str] = None
        self.last_timing = None

    # -- setup --------------------------------------------------------------------------------
    def _layout(self, msgs):
        offs, n = lane_layout(msgs)
        return offs, max(n, self.segment_elems), lane_chunks(msgs, offs, self.chunk_elems)

    def _node(self, r: int) -> Optional[int]:
        if self.numa_nodes is None or not (0 <= r < len(self.numa_nodes)):
            return None
        n = self.numa_nodes[r]
        return int(n) if n is not None and n >= 0 else None

    def create_segments(self) -> None:
        for dst, ms in sorted(self.out_msgs.items()):
            _, n, _ = self._layout(ms)
            self.out_seg[dst] = _Segment(segment_path(self.token, self.rank, dst), n, create=True,
                                         numa_node=self._node(dst))

    def open_segments(self) -> None:
        for src, ms in sorted(self.in_msgs.items()):
            _, n, _ = self._layout(ms)
            self.in_seg[src] = _Segment(segment_path(self.token, src, self.rank), n, create=False)
        from . import _lib
        self._lib = _lib.load()
        if self.gpu:
            from .streams import role_stream
            for seg in list(self.out_seg.values()) + list(self.in_seg.values()):
                seg.register(self._lib)
            # the process's two lane streams (streams.py): every lane of the run shares them
            self.out_stream = role_stream("lane_out", self.device)
            self.in_stream = role_stream("lane_in", self.device)
        pump = ctypes.c_void_p()
        _lib.check("cfa_lane_pump_create", self._lib.cfa_lane_pump_create(
            ctypes.byref(pump), ctypes.c_void_p(self.in_stream.cuda_stream if self.gpu else 0),
            self.device.index if self.gpu else 0, 0 if self.gpu else 1))
        self._pump = pump
        # a lane dropped without close() (an exception, interpreter exit) still stops its pump
        # thread before the HIP runtime goes away
        self._pump_finalizer = weakref.finalize(self, self._lib.cfa_lane_pump_destroy, pump)
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
            lane.close()
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
        # per group: the in-plan index after its last chunk (the plan is sorted by group)
        self._group_end = {}
        for i, x in enumerate(self._in_plan):
            self._group_end[x[0]] = i + 1

    # -- one round -------------------------------------------------------------------------------
    @property
    def elems_out(self) -> int:
        return sum(m.count for ms in self.out_msgs.values() for m in ms)

    @property
    def elems_in(self) -> int:
        return sum(m.count for ms in self.in_msgs.values() for m in ms)

    def check(self) -> None:
        """Raise if a round of this lane has failed (a wait timed out): the lane is unusable."""
        if self._error is not None:
            raise RuntimeError(f"host lane rank {self.rank}: {self._error}")

    def _wait(self, seg: _Segment, word: int, value: int, what: str, r: int) -> None:
        """Host-side wait for ``seg``'s ``word`` to reach ``value``; a timeout fails round ``r``
        here and now, and the lane with it."""
        if _reached(seg.read(word), value):
            return
        from . import _lib
        lib = self._lib or _lib.load()
        rc = lib.cfa_host_wait_word(ctypes.c_void_p(seg.word_host(word)), value & 0xFFFFFFFF,
                                    max(1, int(self.timeout_s * 1e6)))
        if rc == _lib.CFA_OK:
            return
        msg = (f"round {r}: timed out after {self.timeout_s:g} s waiting for {what} (word {seg.read(word)}, "
               f"want {value & 0xFFFFFFFF}); the round's lane rows are invalid")
        if rc != _lib.CFA_E_TIMEOUT:
            msg = f"round {r}: waiting for {what} failed ({_lib.load().cfa_last_error().decode()})"
        self._error = msg
        raise LaneTimeout(f"host lane rank {self.rank}: {msg}")

    def run(self, stream=None, timing: bool = False) -> Dict[int, LaneGate]:
        """Start one round: wait (host) for the ACKs of round r - 2, enqueue every D2H copy and
        its READY signal on the out stream after ``stream``'s earlier work (the rows are final
        before they leave, and the halo rows are no longer read when they are overwritten).
        Finishes the previous round first if its caller did not. Returns {group: LaneGate}.
        ``timing`` records HIP events at the start and end of each stream's work
        (``timing_ms``)."""
        self.check()
        if self._cur is not None:
            self.finish()
        r = self.round
        self.round += 1
        rnd = self._cur = _Round(r, timing and self.gpu)
        par = r & 1
        try:
            if self.gpu:
                st = stream if stream is not None else torch.cuda.current_stream(self.device)
                self.out_stream.wait_stream(st)
                self.in_stream.wait_stream(st)
                if rnd.timing:
                    for k, s in (("o0", self.out_stream), ("i0", self.in_stream)):
                        rnd.ev[k] = torch.cuda.Event(enable_timing=True)
                        rnd.ev[k].record(s)
            if r >= 2:  # the receiver has drained round r - 2 from this parity
                for dst, seg in self.out_seg.items():
                    self._wait(seg, ACK, r - 1, f"rank {dst}'s ack of round {r - 2}", r)
            if self.gpu:
                from . import _lib
                lib, osh = self._lib, ctypes.c_void_p(self.out_stream.cuda_stream)
                for g, dst, k, so, src in self._out_plan:
                    seg = self.out_seg[dst]
                    _lib.check("cfa_memcpy_async", lib.cfa_memcpy_async(
                        ctypes.c_void_p(seg.host_ptr(par, so)), ctypes.c_void_p(src.data_ptr()), src.numel() * 4, osh))
                    seq = (r * self._out_n[dst] + k + 1) & 0xFFFFFFFF
                    _lib.check("cfa_stream_signal", lib.cfa_stream_signal(ctypes.c_void_p(seg.word_dev(READY)), seq,
                                                                          osh))
                if rnd.timing:  # the out stream's work of the round is all enqueued here
                    rnd.ev["o1"] = torch.cuda.Event(enable_timing=True)
                    rnd.ev["o1"].record(self.out_stream)
            else:
                for g, dst, k, so, src in self._out_plan:
                    seg = self.out_seg[dst]
                    n = src.numel()
                    seg.data[par * seg.elems + so: par * seg.elems + so + n].copy_(src)
                    seg.words[READY] = (r * self._out_n[dst] + k + 1) & 0xFFFFFFFF
            self._submit_receive(rnd)
        except LaneTimeout:
            raise
        except Exception as exc:
            self._error = f"round {r}: {type(exc).__name__}: {exc}"
            raise
        return {g: LaneGate(self, rnd, g) for g in self._groups}

    def _event(self, timing: bool):
        """A HIP event the pump records: created (by a first record on the in stream, before the
        round's operations) so that its handle exists and torch knows it was recorded."""
        e = torch.cuda.Event(enable_timing=timing)
        e.record(self.in_stream)
        return e

    def _submit_receive(self, rnd: _Round) -> None:
        """The round's receive side as pump operations: per chunk, wait for its READY number, copy
        it H2D (after the first chunk's wait, a timing event: the pipeline is full), the group's
        event and progress mark after a group's last chunk; then every incoming segment's ACK, and
        the in stream's end event when timed."""
        from . import _lib
        r, par = rnd.r, rnd.r & 1
        ops = []
        for i, (g, src_rank, k, so, dst) in enumerate(self._in_plan):
            seg = self.in_seg[src_rank]
            seq = (r * self._in_n[src_rank] + k + 1) & 0xFFFFFFFF
            op = _lib.LaneOp(wait_word=seg.word_host(READY), wait_value=seq, dst=dst.data_ptr(),
                             src=seg.host_ptr(par, so), bytes=dst.numel() * 4)
            if rnd.timing and i == 0:
                rnd.ev["i_first"] = self._event(True)
                ops.append(_lib.LaneOp(wait_word=seg.word_host(READY), wait_value=seq,
                                       event=rnd.ev["i_first"].cuda_event))
            if self._group_end[g] == i + 1:
                op.mark = i + 1
                if self.gpu:
                    rnd.events[g] = self._event(rnd.timing)
                    op.event = rnd.events[g].cuda_event
            ops.append(op)
        ack = (r + 1) & 0xFFFFFFFF
        for src_rank, seg in self.in_seg.items():
            ops.append(_lib.LaneOp(signal_word=seg.word_dev(ACK) if self.gpu else seg.word_host(ACK),
                                   signal_value=ack))
        if rnd.timing:
            rnd.ev["i1"] = self._event(True)
            ops.append(_lib.LaneOp(event=rnd.ev["i1"].cuda_event))
        rnd.ops = (_lib.LaneOp * len(ops))(*ops)  # alive until the round is finished
        _lib.check("cfa_lane_pump_submit", self._lib.cfa_lane_pump_submit(
            self._pump, ctypes.cast(rnd.ops, ctypes.c_void_p), len(ops), max(1, int(self.timeout_s * 1e6))))

    def _pump_wait(self, mark: int, rnd: _Round, what: str) -> None:
        from . import _lib
        # the pump's own waits time out after timeout_s each; this bound only guards a pump that died
        rc = self._lib.cfa_lane_pump_wait(self._pump, mark, int((4 * self.timeout_s + 60.0) * 1e6))
        if rc == _lib.CFA_OK:
            return
        msg = (f"round {rnd.r}: the lane failed while {what} "
               f"({self._lib.cfa_last_error().decode()}); the round's lane rows are invalid")
        self._error = msg
        raise LaneTimeout(f"host lane rank {self.rank}: {msg}") if rc == _lib.CFA_E_TIMEOUT else \
            RuntimeError(f"host lane rank {self.rank}: {msg}")

    def pump(self) -> None:
        """Kept for callers that interleave it with their mixes: the native pump thread enqueues
        every chunk as it arrives, so there is nothing to do here."""

    def advance(self, group: int, rnd: Optional[_Round] = None):
        """Block (on the host; the GIL is released) until the pump has enqueued every chunk of
        ``group`` and the groups before it; the event after the group's copies (GPU) or None
        (CPU, where the copies are done)."""
        self.check()
        rnd = rnd or self._cur
        if rnd is None:
            raise RuntimeError("host lane: no round in progress")
        if rnd is self._cur and not rnd.done:
            self._pump_wait(self._group_end.get(group, 0), rnd, f"waiting for group {group}")
        return rnd.events.get(group)

    def finish(self) -> None:
        """Complete the current round on the host: wait until the pump has walked all of it (every
        H2D and the ACKs enqueued on the in stream)."""
        rnd = self._cur
        if rnd is None:
            return
        self.check()
        self._pump_wait(-1, rnd, "finishing the round")
        if self.gpu:
            if rnd.timing:
                rnd.ev["groups"] = dict(rnd.events)
            self.last_timing = rnd.ev if rnd.timing else None
        rnd.done = True
        self._cur = None
        self._last_round = rnd

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
        """Finish the round on the host and make ``stream`` wait for its lane work (both
        directions)."""
        self.finish()
        if self.gpu:
            stream.wait_stream(self.out_stream)
            stream.wait_stream(self.in_stream)

    def close(self) -> None:
        """Stop the pump (a round still in progress is abandoned: its peer's next wait times out),
        drain the lane's streams, then unpin and drop the segments."""
        self._cur = None
        if self._pump is not None:
            self._pump_finalizer()  # cfa_lane_pump_destroy, once
            self._pump = None
        if self.gpu and hasattr(self, "out_stream"):
            self.out_stream.synchronize()
            self.in_stream.synchronize()
        for seg in list(self.out_seg.values()) + list(self.in_seg.values()):
            seg.close()
        self.out_seg, self.in_seg = {}, {}

    def pairs(self) -> List[dict]:
        """Every pair this rank sends to: receiver, the NUMA nodes of both GPUs, the node the
        segment's pages were placed on (first, middle, last data page) and why placement was not
        applied, if it was not."""
        out = []
        for dst, seg in sorted(self.out_seg.items()):
            placed = seg.placed_nodes() if seg.mm is not None else []
            out.append({"dst": dst, "src_node": self._node(self.rank), "dst_node": self._node(dst),
                        "placed_nodes": placed, "MB": round(seg.data_bytes / 1e6, 1),
                        **({"numa_note": seg.numa_note} if seg.numa_note else {})})
        return out

    def summary(self) -> dict:
        return {"token": self.token, "chunk_MB": round(self.chunk_elems * 4 / 2**20, 2),
                "out_MB": round(self.elems_out * 4 / 1e6, 2), "in_MB": round(self.elems_in * 4 / 1e6, 2),
                "peers_out": sorted(self.out_msgs), "peers_in": sorted(self.in_msgs),
                "waits": "host (cfa_host_wait_word)", "pairs": self.pairs()}


def new_token() -> str:
    """A job-unique segment-name token (rank 0 draws it; the caller broadcasts it)."""
    return f"{os.getpid()}_{int.from_bytes(os.urandom(4), 'little'):08x}"
