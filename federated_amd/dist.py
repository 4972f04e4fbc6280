"""Cross-shard transports for a simulated device population sharded one shard per GPU.

The reference exchanges neighbour models through files on a shared directory (TF1
``cfa.py:119-130``, TF2 ``consensus_v3.py:82-141``). With the population sharded over the GPUs
of one node, the only cross-shard traffic of a consensus round is the grouped point-to-point
halo exchange of boundary buckets; FedAvg sums map to all-reduce.

Two interchangeable transports:

* ``RcclTransport`` — the MI355X path: an RCCL communicator owned by ``libcfa.so``
  (``cfa_comm_init`` / ``cfa_halo_exchange_f32`` / ``cfa_allreduce_sum_f32``) over xGMI, enqueued
  on a caller-chosen HIP stream so the exchange overlaps interior mixing on another stream.
  The 128-byte unique id is broadcast over the existing ``torch.distributed`` group.
* ``TorchTransport`` — ``torch.distributed`` P2P (``batch_isend_irecv``). With the gloo backend
  this runs the same sharding logic on CPU tensors (multi-process CPU tests).
"""
from __future__ import annotations

import contextlib
import ctypes
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

Transfer = Tuple[torch.Tensor, int]  # (contiguous buffer, peer rank)


class TorchTransport:
    """torch.distributed point-to-point exchange (any backend; gloo for CPU tests)."""

    name = "torch"

    def __init__(self, group=None):
        self.group = group

    @property
    def host_staged(self) -> bool:
        """True on a gloo group: device buffers go through host memory, so an exchange measured on
        this transport says nothing about xGMI (a bench line on it is not comparable)."""
        return dist.get_backend(self.group) == "gloo"

    def exchange(self, sends: Sequence[Transfer], recvs: Sequence[Transfer], stream=None) -> None:
        """Grouped exchange. gloo moves host tensors only, so device buffers are staged through
        host memory, synchronously: the staging copies run on ``stream`` (not on the caller's
        current stream, whose queued mixes they would otherwise wait for), and ``stream`` is
        synchronised before the call returns. With nccl the ops are issued on ``stream``."""
        if not sends and not recvs:
            return
        staged = dist.get_backend(self.group) == "gloo"
        on_dev = staged and stream is not None and any(b.is_cuda for b, _ in list(sends) + list(recvs))
        if staged:
            if on_dev:
                stream.synchronize()
            with torch.cuda.stream(stream) if on_dev else contextlib.nullcontext():
                s_bufs = [(b.cpu() if b.is_cuda else b, p) for b, p in sends]
            r_bufs = [(torch.empty(b.shape, dtype=b.dtype) if b.is_cuda else b, p) for b, p in recvs]
        else:
            s_bufs, r_bufs = list(sends), list(recvs)
        ctx = torch.cuda.stream(stream) if (stream is not None and not staged) else contextlib.nullcontext()
        with ctx:
            ops = [dist.P2POp(dist.isend, b, p, group=self.group) for b, p in s_bufs]
            ops += [dist.P2POp(dist.irecv, b, p, group=self.group) for b, p in r_bufs]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        with torch.cuda.stream(stream) if on_dev else contextlib.nullcontext():
            for (dst, _), (src, _) in zip(recvs, r_bufs):
                if dst is not src:
                    dst.copy_(src)
        if on_dev:
            stream.synchronize()

    def _collective(self, buf: torch.Tensor, stream, fn) -> None:
        """Run ``fn(tensor)`` on ``buf``; gloo moves host tensors only, so a device buffer is
        staged through host memory (synchronously)."""
        if dist.get_backend(self.group) == "gloo" and buf.is_cuda:
            if stream is not None:
                stream.synchronize()
            host = buf.cpu()
            fn(host)
            buf.copy_(host)
            return
        ctx = torch.cuda.stream(stream) if (stream is not None and buf.is_cuda) else contextlib.nullcontext()
        with ctx:
            fn(buf)

    def allreduce_sum(self, buf: torch.Tensor, stream=None) -> None:
        self._collective(buf, stream, lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group))

    def reduce_sum(self, buf: torch.Tensor, root: int, stream=None) -> None:
        """Sum of every rank's ``buf`` into ``buf`` on ``root`` (other ranks' buffers undefined)."""
        self._collective(buf, stream, lambda t: dist.reduce(t, dst=root, op=dist.ReduceOp.SUM, group=self.group))

    def close(self) -> None:
        pass


class RcclTransport:
    """RCCL communicator from libcfa.so (one per process/GPU)."""

    name = "rccl"
    host_staged = False

    def __init__(self, rank: int, world: int, device: int, group=None):
        from . import _lib
        self._lib = _lib
        uid = (ctypes.c_char * _lib.CFA_UNIQUE_ID_BYTES)()
        payload = [None]
        if rank == 0:
            try:
                _lib.call("cfa_comm_unique_id", ctypes.cast(uid, ctypes.c_void_p))
                payload = [bytes(uid)]
            except _lib.CFAError as exc:
                payload = [f"error: {exc}"]
        if world > 1:  # rank 0 always broadcasts (id or failure), so no rank is left waiting
            dist.broadcast_object_list(payload, src=0, group=group)
        if not isinstance(payload[0], bytes):
            raise RuntimeError(f"RCCL unique id unavailable ({payload[0]})")
        ctypes.memmove(uid, payload[0], _lib.CFA_UNIQUE_ID_BYTES)
        comm = ctypes.c_void_p()
        _lib.call("cfa_comm_init", ctypes.byref(comm), rank, world, ctypes.cast(uid, ctypes.c_void_p),
                  int(device))
        self.comm = comm
        self.rank, self.world, self.device = rank, world, device

    @staticmethod
    def _stream(stream) -> int:
        s = stream if stream is not None else torch.cuda.current_stream()
        return int(s.cuda_stream)

    def prepare(self, sends: Sequence[Transfer], recvs: Sequence[Transfer]):
        """Bind one grouped exchange (buffers of any lengths, one message each) to its ctypes
        tables once; returns ``run(stream)``, which enqueues it with one foreign call
        (cfa_p2p_group_f32). The buffers must stay alive and in place."""
        for b, _ in list(sends) + list(recvs):
            if not (b.is_cuda and b.dtype == torch.float32 and b.is_contiguous()):
                raise TypeError("exchange buffers must be contiguous fp32 CUDA tensors")
        # messages to ourselves pair up here, in order: their lengths must agree (a remote pair's
        # lengths are the caller's schedule, e.g. halo.RoutePlan, checked by its digest)
        to_self = [b.numel() for b, p in sends if p == self.rank]
        from_self = [b.numel() for b, p in recvs if p == self.rank]
        if to_self != from_self:
            raise ValueError(f"self messages do not pair up: sends {to_self} vs receives {from_self}")
        L = self._lib
        args = (self.comm, L.ptr_table([b.data_ptr() for b, _ in sends]), L.size_array([b.numel() for b, _ in sends]),
                L.int_array([p for _, p in sends]), len(sends), L.ptr_table([b.data_ptr() for b, _ in recvs]),
                L.size_array([b.numel() for b, _ in recvs]), L.int_array([p for _, p in recvs]), len(recvs))
        keep = (list(sends), list(recvs))

        def run(stream=None):
            L.call("cfa_p2p_group_f32", *args, self._stream(stream))

        run.keep = keep
        return run

    def exchange(self, sends: Sequence[Transfer], recvs: Sequence[Transfer], stream=None) -> None:
        """Enqueue one grouped exchange on ``stream`` (asynchronous): each (buffer, peer) is one
        message of buffer.numel() floats; the caller orders stream dependencies."""
        if not sends and not recvs:
            return
        self.prepare(sends, recvs)(stream)

    def allreduce_sum(self, buf: torch.Tensor, stream=None) -> None:
        """In-place sum all-reduce of a contiguous fp32 device buffer, enqueued on ``stream``."""
        self._check_collective(buf)
        self._lib.call("cfa_allreduce_sum_f32", self.comm, buf.data_ptr(), buf.data_ptr(), buf.numel(),
                       self._stream(stream))

    def reduce_sum(self, buf: torch.Tensor, root: int, stream=None) -> None:
        """In-place sum reduce to ``root``, enqueued on ``stream``."""
        self._check_collective(buf)
        self._lib.call("cfa_reduce_sum_f32", self.comm, buf.data_ptr(), buf.data_ptr(), buf.numel(), int(root),
                       self._stream(stream))

    @staticmethod
    def _check_collective(buf: torch.Tensor) -> None:
        if not (buf.is_cuda and buf.dtype == torch.float32 and buf.is_contiguous()):
            raise TypeError("collective buffers must be contiguous fp32 CUDA tensors")

    def close(self) -> None:
        if self.comm:
            self._lib.call("cfa_comm_destroy", self.comm)
            self.comm = None


def make_transport(kind: str, rank: int, world: int, device: Optional[int] = None, group=None):
    if kind == "rccl":
        return RcclTransport(rank, world, device if device is not None else torch.cuda.current_device(),
                             group)
    if kind == "torch":
        return TorchTransport(group)
    raise ValueError(f"unknown transport {kind!r}")
