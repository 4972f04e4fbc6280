"""Host ingress/egress for buckets that start and end in host memory.

In the reference every neighbour model reaches the mixing step as host numpy arrays: scipy
``.mat`` files (TF1 ``cfa.py:44,60``), pickled ``.npy`` object arrays (TF2
``consensus_v3.py:130``) or MQTT pickles (``learner_consensus.py:136-145``). The engine stages
them through page-locked (pinned) host buffers so H2D/D2H run as async DMA on the copy engines,
and chunks large buckets so copies in both directions overlap the mix of earlier chunks.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .engine import BucketLayout, Engine


class PinnedPool:
    """Re-usable pinned host buffers keyed by element count (no per-call pinning cost)."""

    def __init__(self):
        self._free: Dict[int, List[torch.Tensor]] = {}

    def get(self, n: int) -> torch.Tensor:
        lst = self._free.get(n)
        if lst:
            return lst.pop()
        return torch.empty(n, dtype=torch.float32, pin_memory=True)

    def put(self, t: torch.Tensor) -> None:
        self._free.setdefault(t.numel(), []).append(t)


class DeviceBuckets:
    """Device-resident working set for one device's consensus call: the local bucket, the
    neighbour buckets and the output, re-used across calls of the same shape."""

    def __init__(self, engine: Engine):
        self.engine = engine
        self._bufs: Dict[Tuple[str, int], torch.Tensor] = {}
        self.pool = PinnedPool()

    def buf(self, name: str, P: int) -> torch.Tensor:
        key = (name, P)
        t = self._bufs.get(key)
        if t is None:
            t = self._bufs[key] = self.engine.empty(P)
        return t

    def upload(self, name: str, layout: BucketLayout, arrays, stream=None) -> torch.Tensor:
        """Pack per-layer host arrays into a pinned buffer and copy it to the device (async)."""
        host = self.pool.get(layout.P)
        layout.pack(arrays, host.numpy())
        dev = self.buf(name, layout.P)
        s = stream or torch.cuda.current_stream(self.engine.device)
        with torch.cuda.stream(s):
            dev.copy_(host, non_blocking=True)
        # the pinned buffer may be re-used only after the copy has run
        ev = torch.cuda.Event()
        ev.record(s)
        self._pending = getattr(self, "_pending", [])
        self._pending.append((ev, host))
        return dev

    def download(self, dev: torch.Tensor, stream=None) -> np.ndarray:
        """Copy a device bucket to a fresh host fp32 array (synchronous w.r.t. the host)."""
        s = stream or torch.cuda.current_stream(self.engine.device)
        host = self.pool.get(dev.numel())
        with torch.cuda.stream(s):
            host.copy_(dev, non_blocking=True)
        s.synchronize()
        out = host.numpy().copy()
        self.pool.put(host)
        self.release()
        return out

    def release(self) -> None:
        """Return pinned buffers whose copies have completed to the pool."""
        keep = []
        for ev, host in getattr(self, "_pending", []):
            if ev.query():
                self.pool.put(host)
            else:
                keep.append((ev, host))
        self._pending = keep


def measure_e2e(engine: Engine, P: int, K: int, reps: int = 5, chunks: int = 8) -> dict:
    """Host-resident CFA mix (buckets start and end in pinned host memory): H2D of K+1 buckets,
    mix, D2H of the output. Reports (a) the serial form and (b) a chunked pipeline (chunk-major
    staging, one H2D per chunk) that overlaps H2D of chunk c+1, the mix of chunk c and D2H of
    chunk c-1 on separate streams."""
    dev = engine.device
    host_in = [torch.empty(P, dtype=torch.float32, pin_memory=True).normal_() for _ in range(K + 1)]
    host_out = torch.empty(P, dtype=torch.float32, pin_memory=True)
    d_in = [torch.empty(P, dtype=torch.float32, device=dev) for _ in range(K + 1)]
    d_out = torch.empty(P, dtype=torch.float32, device=dev)
    alphas = [1.0 / (K + 1)] * K
    s = torch.cuda.current_stream(dev)

    def serial():
        for h, d in zip(host_in, d_in):
            d.copy_(h, non_blocking=True)
        engine.mix_seq(d_out, d_in[0], d_in[1:], alphas, s)
        host_out.copy_(d_out, non_blocking=True)

    # Pipelined form: chunk-major pinned staging (chunk c = the K+1 slices [a_c, b_c) back to
    # back), so each chunk is ONE H2D copy; the mix of chunk c waits for its copy, its D2H for
    # the mix, on three streams.
    h2d, k2, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    step = -(-P // chunks)
    step += (-step) % 4
    bounds = [(a, min(a + step, P)) for a in range(0, P, step)]
    pad = lambda m: m + (-m) % 4
    offs, total = [], 0
    for a, b in bounds:
        offs.append(total)
        total += (K + 1) * pad(b - a)
    host_stage = torch.empty(total, dtype=torch.float32, pin_memory=True)
    dev_stage = torch.empty(total, dtype=torch.float32, device=dev)
    for (a, b), o in zip(bounds, offs):
        w = pad(b - a)
        for j, h in enumerate(host_in):
            host_stage[o + j * w:o + j * w + (b - a)].copy_(h[a:b])

    def pipelined():
        for (a, b), o in zip(bounds, offs):
            w = pad(b - a)
            with torch.cuda.stream(h2d):
                dev_stage[o:o + (K + 1) * w].copy_(host_stage[o:o + (K + 1) * w], non_blocking=True)
            k2.wait_stream(h2d)
            src = [dev_stage[o + j * w:o + j * w + (b - a)] for j in range(K + 1)]
            engine.mix_seq(d_out[a:b], src[0], src[1:], alphas, k2)
            d2h.wait_stream(k2)
            with torch.cuda.stream(d2h):
                host_out[a:b].copy_(d_out[a:b], non_blocking=True)

    # Zero-copy form: the mix kernel reads the pinned host buckets over PCIe and writes the
    # pinned host output directly (Engine.mix_seq_pinned): no staging copies, and the write
    # direction of the link overlaps the reads.
    def zero_copy():
        engine.mix_seq_pinned(host_out, host_in[0], host_in[1:], alphas, s)

    res = {}
    for name, fn in (("serial", serial), ("pipelined", pipelined), ("zero_copy", zero_copy)):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / reps
        res[name] = {"ms": round(dt * 1e3, 3),
                     "algorithmic_GBps": round((K + 2) * P * 4 / dt / 1e9, 2),
                     "pcie_bytes": (K + 2) * P * 4}
    # H2D / D2H link rates on their own
    t0 = time.perf_counter()
    for _ in range(reps):
        d_in[0].copy_(host_in[0], non_blocking=True)
    torch.cuda.synchronize(dev)
    res["h2d_GBps"] = round(P * 4 * reps / (time.perf_counter() - t0) / 1e9, 2)
    t0 = time.perf_counter()
    for _ in range(reps):
        host_out.copy_(d_out, non_blocking=True)
    torch.cuda.synchronize(dev)
    res["d2h_GBps"] = round(P * 4 * reps / (time.perf_counter() - t0) / 1e9, 2)
    # each host-resident form against the serial one (copies in, device-resident mix, copy out)
    serial()
    torch.cuda.synchronize(dev)
    ref = host_out.clone()
    for name, fn in (("pipelined", pipelined), ("zero_copy", zero_copy)):
        host_out.zero_()
        fn()
        torch.cuda.synchronize(dev)
        res[f"{name}_equals_device_result"] = bool(torch.equal(host_out, ref))
    return res
