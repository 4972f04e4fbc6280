"""Shared runtime of the drop-in ``consensus`` modules.

* The reference's exchange protocol: polling for neighbour files with ``pause(1)``, one retry
  after ``pause(3)`` when a load fails, and the fixed protocol sleeps (``pause(2)``/``pause(5)``
  around each neighbour). ``pause`` here sleeps ``seconds * FEDERATED_AMD_PAUSE_SCALE``
  (default 1.0 = the reference's timing; set 0 to drop the protocol sleeps).
* ``HostMixer``: the host-array front end of the GPU engine. Per call it flattens the caller's
  per-layer arrays into one pinned staging bucket per model (layer order kept) and runs ONE
  libcfa kernel that folds all n neighbours (plus the optional fused compression epilogue).
  By default the kernel reads the pinned rows and writes the pinned result in place over PCIe
  (zero-copy: ``SINGLE_ZERO_COPY`` for fp32, ``TF1_ZERO_COPY`` for the fp64 TF1 buckets);
  switched off, the buckets move by one H2D and one D2H copy instead. Large mixes take a
  chunk pipeline. There is no CPU fallback: without a GPU the engine raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import _lib, matfile
from ..engine import BucketLayout, get_engine


def _scale() -> float:
    try:
        return float(os.environ.get("FEDERATED_AMD_PAUSE_SCALE", "1"))
    except ValueError:
        return 1.0


def pause(seconds: float) -> None:
    """matplotlib.pyplot.pause(seconds) as the reference uses it: a protocol sleep."""
    s = float(seconds) * _scale()
    if s > 0:
        time.sleep(s)


def wait_for(*paths: str) -> float:
    """Poll until every path exists (cfa.py:120-124: ``pause(1)`` between checks). Returns the
    time spent waiting."""
    t0 = time.time()
    while not all(os.path.isfile(p) for p in paths):
        pause(1)
        if _scale() == 0:
            time.sleep(0.01)
    return time.time() - t0


def loadmat_retry(path: str) -> dict:
    """loadmat with the reference's single retry after pause(3) (cfa.py:43-48). Read by libcfa's
    level-5 codec (federated_amd/matfile.py: scipy.io.loadmat's result, ≈3x faster)."""
    try:
        return matfile.loadmat(path)
    except Exception:
        print("Detected problem while loading file")
        pause(3)
        return matfile.loadmat(path)


def savemat_retry(path: str, data: dict) -> None:
    """savemat with the reference's single retry after pause(3) (cfa.py:131-139). Written by
    libcfa's level-5 codec (federated_amd/matfile.py: scipy.io.savemat's bytes, ≈2.7x faster)."""
    try:
        matfile.savemat(path, data)
    except Exception:
        print("Unable to save file .. retrying")
        pause(3)
        matfile.savemat(path, data)


def _check_coefficients(n: int, alphas, divisors=None) -> None:
    """One coefficient (and divisor) per neighbour: the C entry points read exactly n of each,
    so a short list would be read past its end."""
    if len(alphas) != n:
        raise ValueError(f"one alpha per neighbour required ({len(alphas)} alphas, {n} neighbours)")
    if divisors is not None and len(divisors) != n:
        raise ValueError(f"one divisor per neighbour required ({len(divisors)} divisors, {n} neighbours)")


_layouts: dict = {}
_F32 = np.dtype(np.float32)


def _dtype(a):
    """dtype of an array-like (ndarray fast path)."""
    return a.dtype if isinstance(a, np.ndarray) else np.asarray(a).dtype


def _layout_of(arrays) -> BucketLayout:
    """BucketLayout of the arrays' shapes, cached per shape tuple (building one costs tens of
    microseconds of numpy calls, which a per-call drop-in path cannot afford)."""
    key = tuple([a.shape if type(a) is np.ndarray else np.shape(a) for a in arrays])
    lay = _layouts.get(key)
    if lay is None:
        if len(_layouts) >= 64:
            _layouts.clear()
        lay = _layouts[key] = BucketLayout(key)
    return lay


NATIVE_PIPELINE = True            # fp32 host mixes above NATIVE_MIN_BYTES of staging: cfa_host_mix_f32
NATIVE_MIN_BYTES = 1 << 20        # staging bytes from which the native chunk pipeline beats single-shot
NATIVE_CHUNK_ELEMS = 128 << 10    # elements per model per native pipeline chunk
NATIVE_THREADS = 0                # host copy threads of the native pipeline (0: torch.get_num_threads(), <= 4)
PIPELINE_MIN_BYTES = 64 << 20     # (NATIVE_PIPELINE off) host mixes above this take the Python chunk pipeline
PIPELINE_CHUNK_BYTES = 128 << 20  # staging bytes per pipeline chunk
PIPELINE_ZERO_COPY = True          # pipeline chunks mixed in place in pinned host memory (no H2D/D2H)
SINGLE_ZERO_COPY = True            # single-shot fp32 mixes read/write pinned staging in place (no H2D/D2H)
TF1_ZERO_COPY = True               # TF1 fp64 mixes read/write pinned staging in place (counter stays on device)
SIGNAL_COMPLETION = True           # zero-copy calls end on a GPU-set pinned word, not hipStreamSynchronize
SIGNAL_SPIN_US = 2000              # host spin on that word before falling back to hipStreamSynchronize


class HostMixer:
    """Host arrays in, host arrays out; the arithmetic runs in libcfa on the GPU."""

    def __init__(self, device=None):
        self.engine = get_engine(device)
        self._tls = threading.local()

    def _stream(self) -> torch.cuda.Stream:
        s = getattr(self._tls, "stream", None)
        if s is None:
            s = self._tls.stream = torch.cuda.Stream(self.engine.device)
        return s

    def _upload(self, layout: BucketLayout, arrays) -> torch.Tensor:
        host = torch.from_numpy(layout.pack(arrays))
        return host.to(self.engine.device, non_blocking=False)

    def _cached(self, kind: str, n: int, dtype=torch.float32, pinned: bool = False) -> torch.Tensor:
        """Per-thread cached staging buffer (pinned host or device) of at least n elements."""
        cache = getattr(self._tls, "bufs", None)
        if cache is None:
            cache = self._tls.bufs = {}
        t = cache.get((kind, dtype))
        if t is None or t.numel() < n:
            if pinned:
                t = torch.empty(max(n, 1), dtype=dtype, pin_memory=True)
            else:
                t = torch.empty(max(n, 1), dtype=dtype, device=self.engine.device)
            cache[(kind, dtype)] = t
        return t[:n]

    def mix(self, local: Sequence, nbrs: Sequence[Sequence], alphas: Sequence[float],
            compress: Optional[Tuple[int, int]] = None,
            divisors: Optional[Sequence[float]] = None,
            tf1: bool = False) -> Tuple[List[np.ndarray], Optional[int]]:
        """Sequential CFA mix of the per-layer arrays ``local`` with each neighbour's per-layer
        arrays, w <- w + alphas[j] * (x_j - w) per layer, all n neighbours folded in one kernel.
        ``compress=(mode, layer)`` fuses the cfa_ongraphs compression epilogue on that layer
        (with the pre-mix local as DPCM reference) and returns the kept count.
        ``divisors`` selects the FedAvg form w <- w + (alphas[j] * (x_j - w)) / divisors[j].
        ``tf1`` selects the TF1 numerics (``cfa_mix_tf1_f32``): ``alphas`` are the float64
        products eps * wf_j, the chain and the epilogue run in fp64 as the reference's do under
        numpy 2, and the result is that fp64 result rounded once to fp32.

        Host path: the local and all neighbour buckets are packed into ONE cached
        pinned staging buffer (rows padded to 16-byte pitch). By default (``SINGLE_ZERO_COPY``)
        the kernel reads those rows over PCIe in place and writes the result into pinned host
        memory: no staging copies, one stream synchronisation; a compression count stays on the
        device and returns by one 8-byte copy. With ``SINGLE_ZERO_COPY = False`` the staging
        moves by one async H2D copy and the result by one D2H (same kernels, same results).
        Returns (fp32 arrays with the local shapes, kept count or None).

        From NATIVE_MIN_BYTES of staging (without compression or the TF1 rule) the whole host path
        runs as libcfa's chunk pipeline ``_mix_native`` instead (pack / PCIe kernel / unpack
        overlapped chunk by chunk in one call; same kernels per chunk, same results); with
        ``NATIVE_PIPELINE = False`` buckets above PIPELINE_MIN_BYTES take the Python pipeline
        ``_mix_pipelined``."""
        layout = _layout_of(local)
        P, n = layout.P, len(nbrs)
        _check_coefficients(n, alphas, divisors)
        if not tf1 and compress is None and n > 0:
            if NATIVE_PIPELINE and (n + 1) * P * 4 >= NATIVE_MIN_BYTES:
                return self._mix_native(layout, local, nbrs, alphas, divisors), None
            if (n + 1) * P * 4 >= PIPELINE_MIN_BYTES:
                return self._mix_pipelined(layout, local, nbrs, alphas, divisors), None
        st = self._stream()
        if SINGLE_ZERO_COPY:
            return self._mix_zero_copy(layout, local, nbrs, alphas, divisors, st, compress, tf1)
        with torch.cuda.stream(st):
            host = self._cached("h_in", (n + 1) * P, pinned=True)
            hv = host.numpy().reshape(n + 1, P)
            layout.pack(local, hv[0])
            for j, x in enumerate(nbrs):
                layout.pack(x, hv[j + 1])
            dev = self._cached("d_in", (n + 1) * P)
            dev.copy_(host, non_blocking=True)
            d = dev.view(n + 1, P)
            out = self._cached("d_out", P)
            kept = None
            if tf1:
                mode, b, e = 0, 0, 0
                if compress is not None:
                    mode, layer = compress
                    b, e = layout.segment(layer)
                    kept = self._cached("d_cnt", 1, torch.int64)
                    kept.zero_()
                self.engine.mix_tf1(out, d[0], list(d[1:]), [float(a) for a in alphas], mode, b, e, kept,
                                    stream=st)
            elif compress is not None:
                mode, layer = compress
                b, e = layout.segment(layer)
                kept = self._cached("d_cnt", 1, torch.int64)
                kept.zero_()
                self.engine.mix_seq_compress(out, d[0], list(d[1:]), list(alphas), mode, b, e, kept, stream=st)
            elif divisors is not None:
                self.engine.mix_seq_div(out, d[0], list(d[1:]), list(alphas), list(divisors), stream=st)
            else:
                self.engine.mix_seq(out, d[0], list(d[1:]), list(alphas), stream=st)
            h_out = self._cached("h_out", P, pinned=True)
            h_out.copy_(out, non_blocking=True)
            if kept is not None:
                h_cnt = self._cached("h_cnt", 1, torch.int64, pinned=True)
                h_cnt.copy_(kept, non_blocking=True)
            st.synchronize()
            flat = h_out.numpy().copy()  # the pinned buffer is reused by the next call
            kept_n = int(h_cnt.numpy()[0]) if kept is not None else None
        return layout.unpack(flat, copy=False), kept_n

    def _zc_plan(self, kind: str, layout: BucketLayout, n: int, dtype, out_dtype=None) -> "_ZeroCopyPlan":
        """Per-thread cached zero-copy plan for one (kind, layout, fan-in): pinned rows and
        output, their device addresses and the ctypes tables, built once. ``layout`` is a cached
        ``_layout_of`` object, so it identifies the layer shapes."""
        plans = getattr(self._tls, "plans", None)
        if plans is None:
            plans = self._tls.plans = {}
        key = (kind, id(layout), n)
        plan = plans.get(key)
        if plan is None or plan.layout is not layout:
            if len(plans) >= 16:  # bounded: drop the oldest layout
                plans.pop(next(iter(plans)))
            plan = plans[key] = _ZeroCopyPlan(self, layout, n, dtype, out_dtype,
                                              counter=kind not in ("mewma64", "fold64"))
        return plan

    def _mix_zero_copy(self, layout: BucketLayout, local, nbrs, alphas, divisors, st,
                       compress=None, tf1=False) -> Tuple[List[np.ndarray], Optional[int]]:
        """Single-shot fp32 mix without staging copies: the buckets are packed into pinned rows
        (pitch rounded up to 4 elements, so every row stays 16-byte aligned), the kernel reads
        them over PCIe and writes the result into pinned host memory; one synchronisation. The
        compression count (device atomics) stays in device memory and returns by one 8-byte
        copy (cfa_counter_fetch, which also re-zeroes it). Everything but the pack, the launch
        and the unpack is prepared once per layout (``_ZeroCopyPlan``)."""
        n = len(nbrs)
        plan = self._zc_plan("f32", layout, n, np.float32)
        plan.pack(local, nbrs)
        sh = plan.stream_handle(st)
        lib = plan.lib
        if tf1 or compress is not None:
            mode, b, e = 0, 0, 0
            if compress is not None:
                mode, layer = compress
                b, e = layout.segment(layer)
                if not (0 <= b <= e <= plan.P):
                    raise ValueError("bad compression layer")
            kp = plan.counter if compress is not None else None
            if tf1:
                rc = lib.cfa_mix_tf1_f32(plan.ob, plan.hb, plan.table, plan.coeffs(alphas, True), n, plan.P,
                                         int(mode), int(b), int(e), kp, sh)
                name = "cfa_mix_tf1_f32"
            else:
                rc = lib.cfa_mix_seq_compress_f32(plan.ob, plan.hb, plan.table, plan.coeffs(alphas), n, plan.P,
                                                  int(mode), int(b), int(e), kp, sh)
                name = "cfa_mix_seq_compress_f32"
        elif divisors is not None:
            rc = lib.cfa_mix_seq_div_f32(plan.ob, plan.hb, plan.table, plan.coeffs(alphas),
                                         _lib.float_array(list(divisors)), n, plan.P, sh)
            name = "cfa_mix_seq_div_f32"
        else:
            rc = lib.cfa_mix_seq_f32(plan.ob, plan.hb, plan.table, plan.coeffs(alphas), n, plan.P, sh)
            name = "cfa_mix_seq_f32"
        if rc != _lib.CFA_OK and compress is not None:
            plan.reset_count()
        _lib.check(name, rc)
        if compress is not None:
            plan.fetch_count(sh)
        plan.complete(sh)
        kept_n = int(plan.count_host[0]) if compress is not None else None
        return plan.unpack(), kept_n

    def _aux_streams(self):
        s = getattr(self._tls, "aux", None)
        if s is None:
            dev = self.engine.device
            s = self._tls.aux = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
        return s

    def _mix_native(self, layout: BucketLayout, local, nbrs, alphas, divisors,
                    chunk_elems: Optional[int] = None, threads: Optional[int] = None) -> List[np.ndarray]:
        """The whole host path in one libcfa call (``cfa_host_mix_f32``): chunk c of every model
        is copied into pinned staging by a pool of host threads while the zero-copy kernel of
        chunk c - 1 reads over PCIe, and each chunk's result is copied into the output layers
        as soon as it lands. Same kernels per chunk as the single-shot mix, same results."""
        P, n, L = layout.P, len(nbrs), len(layout.sizes)
        chunk = int(chunk_elems or NATIVE_CHUNK_ELEMS)
        nthreads = int(threads or NATIVE_THREADS or min(4, torch.get_num_threads()))
        keep, ins = [], (ctypes.c_void_p * ((n + 1) * L))()
        for m, model in enumerate((local, *nbrs)):
            if len(model) != L:
                raise ValueError(f"expected {L} tensors, got {len(model)}")
            for k, a in enumerate(model):
                a = np.asarray(a)
                if a.dtype != np.float32 or not a.flags.c_contiguous:
                    a = np.ascontiguousarray(a, dtype=np.float32)
                if a.size != layout.sizes[k]:
                    raise ValueError(f"tensor {k} has {a.size} elements, layout expects {layout.sizes[k]}")
                keep.append(a)
                ins[m * L + k] = a.ctypes.data
        outs = [np.empty(shp, dtype=np.float32) for shp in layout.shapes]
        optr = (ctypes.c_void_p * L)(*[o.ctypes.data for o in outs])
        sizes = (ctypes.c_size_t * L)(*layout.sizes)
        need = self.engine.lib.cfa_host_mix_staging_elems(sizes, L, n, chunk)
        staging = self._cached("h_native", need, pinned=True)
        h_out = self._cached("h_out", P, pinned=True)
        a_arr = _lib.float_array(list(alphas))
        d_arr = _lib.float_array(list(divisors)) if divisors is not None else None
        _lib.call("cfa_host_mix_f32", optr, ins, sizes, L, n, a_arr, d_arr, staging.data_ptr(), need,
                  h_out.data_ptr(), chunk, nthreads, self.engine.stream_handle(self._stream()))
        del keep
        return outs

    def _mix_pipelined(self, layout: BucketLayout, local, nbrs, alphas, divisors) -> List[np.ndarray]:
        """Large host-resident mix as a chunk pipeline over three streams. Staging is
        chunk-major: chunk c holds the n + 1 slices [a_c, b_c) of every bucket back to back
        (each padded to a multiple of 4 elements, so every slice stays 16-byte aligned), so each
        chunk is ONE H2D copy. The host packs chunk c + 1 (torch's parallel copy) while chunk c
        is in flight; the mix of chunk c waits for its copy; its D2H waits for the mix."""
        P, n = layout.P, len(nbrs)
        C = max(2, min(32, -(-(n + 1) * P * 4 // PIPELINE_CHUNK_BYTES)))
        step = -(-P // C)
        step += (-step) % 4
        bounds = [(a, min(a + step, P)) for a in range(0, P, step)]
        pad = lambda m: m + (-m) % 4
        offs, total = [], 0
        for a, b in bounds:
            offs.append(total)
            total += (n + 1) * pad(b - a)
        h2d, d2h = self._aux_streams()
        comp = self._stream()
        host = self._cached("h_pipe", total, pinned=True)
        h_out = self._cached("h_out", P, pinned=True)
        zero_copy = PIPELINE_ZERO_COPY
        if zero_copy:  # the kernel reads the packed chunk and writes the result in host memory
            hbase, obase = self.engine.host_device_ptr(host), self.engine.host_device_ptr(h_out)
            a_arr = _lib.float_array(list(alphas))
            d_arr = _lib.float_array(list(divisors)) if divisors is not None else None
        else:
            dev = self._cached("d_pipe", total)
            d_out = self._cached("d_out", P)
        models = [local] + list(nbrs)
        flat = [[torch.from_numpy(np.ascontiguousarray(np.asarray(t)).reshape(-1)) for t in m] for m in models]
        seg = [layout.segment(k) for k in range(len(layout.sizes))]
        outs = [np.empty(shp, dtype=np.float32) for shp in layout.shapes]
        out_flat = [torch.from_numpy(o.reshape(-1)) for o in outs]

        def pieces(a, b):  # (layer k, [x, y) global, [x - lo, y - lo) within the layer)
            for k, (lo, hi) in enumerate(seg):
                x, y = max(a, lo), min(b, hi)
                if x < y:
                    yield k, x, y, lo

        def unpack(c):
            a, b = bounds[c]
            done[c].synchronize()
            for k, x, y, lo in pieces(a, b):
                out_flat[k][x - lo:y - lo].copy_(h_out[x:y])

        def prefault(c):  # first touch of the fresh output pages, off the critical path
            a, b = bounds[c]
            for k, x, y, lo in pieces(a, b):
                out_flat[k][x - lo:y - lo].zero_()

        done, unpacked = [], 0
        for c, ((a, b), o) in enumerate(zip(bounds, offs)):
            w = pad(b - a)
            for j in range(n + 1):  # pack chunk c of every bucket (parallel copies)
                base = o + j * w
                for k, x, y, lo in pieces(a, b):
                    host[base + x - a:base + y - a].copy_(flat[j][k][x - lo:y - lo])
            if zero_copy:
                table = _lib.ptr_table([hbase + 4 * (o + j * w) for j in range(1, n + 1)])
                args = (obase + 4 * a, hbase + 4 * o, table, a_arr)
                sh = self.engine.stream_handle(comp)
                if divisors is not None:
                    _lib.call("cfa_mix_seq_div_f32", *args, d_arr, n, b - a, sh)
                else:
                    _lib.call("cfa_mix_seq_f32", *args, n, b - a, sh)
                ev = torch.cuda.Event()
                ev.record(comp)
            else:
                with torch.cuda.stream(h2d):
                    dev[o:o + (n + 1) * w].copy_(host[o:o + (n + 1) * w], non_blocking=True)
                comp.wait_stream(h2d)
                src = [dev[o + j * w:o + j * w + (b - a)] for j in range(n + 1)]
                if divisors is not None:
                    self.engine.mix_seq_div(d_out[a:b], src[0], src[1:], list(alphas), list(divisors), stream=comp)
                else:
                    self.engine.mix_seq(d_out[a:b], src[0], src[1:], list(alphas), stream=comp)
                d2h.wait_stream(comp)
                with torch.cuda.stream(d2h):
                    h_out[a:b].copy_(d_out[a:b], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(d2h)
            done.append(ev)
            # host work while this chunk's H2D is in flight: fault in this chunk's output pages,
            # and unpack whatever result chunks have already landed (never block on a D2H: the
            # copy queue may order it behind the in-flight H2D)
            prefault(c)
            while unpacked < c and done[unpacked].query():
                unpack(unpacked)
                unpacked += 1
        while unpacked < len(bounds):
            unpack(unpacked)
            unpacked += 1
        return outs

    def compress(self, y: np.ndarray, ref: Optional[np.ndarray], mode: int) -> Tuple[np.ndarray, int]:
        """Standalone compression epilogue (cfa_ongraphs.py:225-273) on one tensor."""
        layout = BucketLayout([np.shape(y)])
        with torch.cuda.stream(self._stream()):
            dy = self._upload(layout, [y])
            dr = self._upload(layout, [ref]) if ref is not None else None
            kept = self.engine.counter()
            self.engine.compress(dy, dr, mode, kept, stream=self._stream())
            flat = dy.cpu().numpy()
            n = int(kept.item())
        return flat.reshape(np.shape(y)), n

    def mewma(self, W: Sequence, states: Sequence[np.ndarray], grads: Sequence[Sequence], rho: float,
              lrs: Sequence[float], init: bool, use_filtered: bool) -> List[np.ndarray]:
        """CFA-GE update of the per-layer model ``W`` with the neighbours' slot gradients
        ``grads[j]`` (per-layer arrays) and the per-layer saved-state arrays ``states[k]`` of shape
        [..., N] (updated IN PLACE at slot j, as the reference does). ``lrs`` = per-layer learning
        rate; layers with the first rate must precede the others (layer 1 then layer 2)."""
        layout = _layout_of(W)
        n = len(grads)
        first_other = next((k for k in range(len(lrs)) if lrs[k] != lrs[0]), len(lrs))
        if any(lr != lrs[-1] for lr in lrs[first_other:]):
            raise ValueError("learning rates must be one value for the leading layers, one for the rest")
        split = int(layout.offsets[first_other])
        lr1, lr2 = float(lrs[0]), float(lrs[-1])
        with torch.cuda.stream(self._stream()):
            dW = self._upload(layout, W)
            ds = [self._upload(layout, [np.asarray(st)[..., j] for st in states]) for j in range(n)]
            dg = [self._upload(layout, g) for g in grads]
            self.engine.mewma(dW, ds, dg, rho, lr1, lr2, split, init, use_filtered,
                              stream=self._stream())
            W_out = dW.cpu().numpy()
            s_out = [x.cpu().numpy() for x in ds]
        for j in range(n):
            for k, arr in enumerate(layout.unpack(s_out[j], copy=False)):
                states[k][..., j] = arr
        return layout.unpack(W_out, copy=False)

    # -- TF1 on fp64 buckets: the reference's own arithmetic and dtypes -----------------------
    @staticmethod
    def _runs(flags):
        """Maximal runs of consecutive tensors sharing a flag: [(first, last + 1, flag)]."""
        runs, k = [], 0
        while k < len(flags):
            e = k
            while e < len(flags) and flags[e] == flags[k]:
                e += 1
            runs.append((k, e, flags[k]))
            k = e
        return runs

    def _upload64(self, layout: BucketLayout, arrays) -> torch.Tensor:
        host = torch.from_numpy(layout.pack(arrays, np.empty(layout.P, dtype=np.float64)))
        return host.to(self.engine.device, non_blocking=False)

    def mix_tf1(self, local: Sequence, nbrs: Sequence[Sequence], alphas: Sequence[float],
                compress: Optional[Tuple[int, int]] = None) -> Tuple[List[np.ndarray], Optional[int]]:
        """TF1 mix with the reference's numerics and dtypes (``cfa_mix_tf1_f64``): the arrays are
        widened to fp64 buckets (exact), folded as numpy 2 folds them (``eps * wf`` is an
        np.float64: fp32 first subtraction when both operands are fp32 arrays, fp64 after), the
        compression epilogue of ``compress=(mode, layer)`` applied in fp64; returns the fp64
        arrays the reference returns, with the local shapes, and the kept count (or None).
        Needs at least one neighbour (with none, the reference returns the inputs themselves)."""
        n = len(nbrs)
        if n == 0:
            raise ValueError("mix_tf1 needs at least one neighbour model")
        _check_coefficients(n, alphas)
        layout = _layout_of(local)
        P = layout.P
        st = self._stream()
        if TF1_ZERO_COPY:  # fp32 arrays (what TF hands the drivers) take one wide launch
            res = self._mix_tf1_wide(layout, local, nbrs, alphas, compress, st)
            if res is not None:
                return res
        first = nbrs[0]
        flags = tuple(_dtype(local[k]) == _F32 and not callable(first) and _dtype(first[k]) == _F32
                      for k in range(len(local)))
        if TF1_ZERO_COPY:
            return self._mix_tf1_zero_copy(layout, local, nbrs, alphas, compress, flags, st)
        with torch.cuda.stream(st):
            host = self._cached("h_in64", (n + 1) * P, torch.float64, pinned=True)
            hv = host.numpy().reshape(n + 1, P)
            layout.pack(local, hv[0])
            for j, x in enumerate(nbrs):
                if callable(x):  # a filler writes the flat bucket itself (e.g. a payload decoder)
                    x(hv[j + 1])
                else:
                    layout.pack(x, hv[j + 1])
            h_out = self._cached("h_out64", P, torch.float64, pinned=True)
            dev = self._cached("d_in64", (n + 1) * P, torch.float64)
            dev.copy_(host, non_blocking=True)
            d = dev.view(n + 1, P)
            out = self._cached("d_out64", P, torch.float64)
            mode, cb, ce, kept = 0, 0, 0, None
            if compress is not None:
                mode, layer = compress
                cb, ce = layout.segment(layer)
                kept = self._cached("d_cnt", 1, torch.int64)
                kept.zero_()
            for k0, k1, f32 in self._runs(flags):  # one launch per run of equal step-0 precision
                b, e = layout.segment(k0)[0], layout.segment(k1 - 1)[1]
                lo, hi = max(cb, b), min(ce, e)
                hit = kept is not None and lo < hi
                self.engine.mix_tf1_f64(out[b:e], d[0, b:e], [d[j, b:e] for j in range(1, n + 1)],
                                        [float(a) for a in alphas], f32, mode if hit else 0,
                                        lo - b if hit else 0, hi - b if hit else 0,
                                        kept if hit else None, stream=st)
            h_out.copy_(out, non_blocking=True)
            if kept is not None:
                h_cnt = self._cached("h_cnt", 1, torch.int64, pinned=True)
                h_cnt.copy_(kept, non_blocking=True)
            st.synchronize()
            flat = h_out.numpy().copy()
            kept_n = int(h_cnt.numpy()[0]) if kept is not None else None
        return layout.unpack(flat, copy=False), kept_n

    def _mix_tf1_wide(self, layout, local, nbrs, alphas, compress, st):
        """mix_tf1 when every array is fp32 (what TF hands the TF1 drivers): fp32 pinned rows, one
        cfa_mix_tf1_wide_f32 launch writing the unrounded fp64 result into a pinned fp64 row.
        Returns None, launching nothing, when the pack meets an array that is not fp32.
        The same values as the fp64-row path (fp32 values widen exactly; step 0 is the fp32
        subtraction there too) at half the packed and PCIe-read bytes."""
        n = len(nbrs)
        plan = self._zc_plan("tf1w", layout, n, np.float32, out_dtype=np.float64)
        if not plan.pack(local, nbrs, require=_F32):
            return None  # some array is not fp32 (or a filler): the fp64-row path takes it
        sh = plan.stream_handle(st)
        mode, cb, ce = 0, 0, 0
        if compress is not None:
            mode, layer = compress
            cb, ce = layout.segment(layer)
        rc = plan.lib.cfa_mix_tf1_wide_f32(plan.ob, plan.hb, plan.table, plan.coeffs(alphas, True), n, plan.P,
                                           int(mode), int(cb), int(ce),
                                           plan.counter if compress is not None else None, sh)
        if rc != _lib.CFA_OK and compress is not None:
            plan.reset_count()
        _lib.check("cfa_mix_tf1_wide_f32", rc)
        if compress is not None:
            plan.fetch_count(sh)
        plan.complete(sh)
        kept_n = int(plan.count_host[0]) if compress is not None else None
        return plan.unpack(), kept_n

    def _mix_tf1_zero_copy(self, layout, local, nbrs, alphas, compress, flags, st):
        """mix_tf1 on pinned fp64 rows read and written in place by the kernel (rows of an even
        number of fp64, so 16-byte aligned for odd P too); one launch per run of layers with
        the same step-0 precision; the compression count comes back by one 8-byte copy."""
        n = len(nbrs)
        plan = self._zc_plan("f64", layout, n, np.float64)
        plan.pack(local, nbrs)
        sh = plan.stream_handle(st)
        mode, cb, ce = 0, 0, 0
        if compress is not None:
            mode, layer = compress
            cb, ce = layout.segment(layer)
        coeffs = plan.coeffs(alphas, True)
        for k0, k1, f32 in plan.runs(flags):
            b, e = layout.segment(k0)[0], layout.segment(k1 - 1)[1]
            lo, hi = max(cb, b), min(ce, e)
            hit = compress is not None and lo < hi
            rc = plan.lib.cfa_mix_tf1_f64(plan.ob + 8 * b, plan.hb + 8 * b, plan.run_table(b), coeffs, n,
                                          int(bool(f32)), e - b, mode if hit else 0, lo - b if hit else 0,
                                          hi - b if hit else 0, plan.counter if hit else None, sh)
            if rc != _lib.CFA_OK:
                plan.lib.cfa_stream_synchronize(sh)  # earlier runs may still read the pinned rows
                if compress is not None:
                    plan.reset_count()
            _lib.check("cfa_mix_tf1_f64", rc)
        if compress is not None:
            plan.fetch_count(sh)
        plan.complete(sh)
        kept_n = int(plan.count_host[0]) if compress is not None else None
        return plan.unpack(), kept_n

    def _mewma_tf1_zero_copy(self, layout, W, states, grads, rho, lr1, lr2, split, init, use_filtered, flags,
                             st) -> List[np.ndarray]:
        """mewma_tf1 on pinned fp64 rows updated in place by the kernel over PCIe (row 0 = W,
        rows 1..n = the saved states' slots, rows n+1..2n = the gradients); one launch per run
        of layers with equal dtype flags; the states are written back into the caller's arrays
        at their slots. Returns the W arrays (fp64)."""
        n = len(grads)
        layout = _layout_of(W) if layout is None else layout
        plan = self._zc_plan("mewma64", layout, 2 * n, np.float64)
        rows = plan.rows
        sizes = layout.sizes
        plan.pack(W, [])  # row 0 (the remaining rows are filled below)
        for j in range(n):
            for k, v in enumerate(plan.views[1 + j]):
                np.copyto(v, np.asarray(states[k])[..., j].reshape(-1), casting="unsafe")
            g = grads[j]
            for k, v in enumerate(plan.views[1 + n + j]):
                a = np.asarray(g[k])
                if a.size != sizes[k]:
                    raise ValueError(f"gradient {j} tensor {k} has {a.size} elements, layout expects {sizes[k]}")
                np.copyto(v, a.reshape(-1), casting="unsafe")
        sh = plan.stream_handle(st)
        ones = plan.strides_one()
        for k0, k1, mask in plan.runs(tuple(flags)):
            b, e = layout.segment(k0)[0], layout.segment(k1 - 1)[1]
            rc = plan.lib.cfa_mewma_tf1_f64(plan.hb + 8 * b, plan.row_table(1, n, b), plan.row_table(1 + n, n, b),
                                            ones, n, float(rho), float(lr1), float(lr2), max(0, min(split, e) - b),
                                            int(bool(init)), int(bool(use_filtered)), int(mask), e - b, sh)
            if rc != _lib.CFA_OK:
                plan.lib.cfa_stream_synchronize(sh)  # earlier runs may still update the pinned rows
            _lib.check("cfa_mewma_tf1_f64", rc)
        plan.complete(sh)
        for j in range(n):
            for k, v in enumerate(plan.views[1 + j]):
                states[k][..., j] = v.reshape(layout.shapes[k])
        P = layout.P
        flat = rows[0, :P].copy()
        return [flat[b:e].reshape(shp) for (b, e), shp in
                zip((layout.segment(k) for k in range(len(sizes))), layout.shapes)]

    def fold64(self, local: Sequence, nbrs: Sequence[Sequence], alphas: Sequence[float], rule: int,
               divisors: Optional[Sequence[float]] = None) -> List[np.ndarray]:
        """fp64 fold (``cfa_fold_f64``) of per-layer arrays widened to fp64 buckets; returns fp64
        arrays with the local shapes. By default (``TF1_ZERO_COPY``) the kernel reads the pinned
        rows and writes the pinned output in place; otherwise one H2D of all buckets, one launch,
        one D2H. A neighbour
        may be given as a callable ``fill(dst)`` that writes its flat fp64 bucket into the pinned
        staging row ``dst`` (the MQTT payload decoder does)."""
        layout = _layout_of(local)
        P, n = layout.P, len(nbrs)
        _check_coefficients(n, alphas, divisors if rule == _lib.RULE_SEQUENTIAL_DIV else None)
        st = self._stream()
        if TF1_ZERO_COPY:  # the kernel reads the pinned fp64 rows and writes the pinned output in place
            plan = self._zc_plan("fold64", layout, n, np.float64)
            plan.pack(local, nbrs)
            sh = plan.stream_handle(st)
            div = _lib.double_array([float(x) for x in divisors]) if divisors is not None else None
            _lib.check("cfa_fold_f64", plan.lib.cfa_fold_f64(plan.ob, plan.hb, plan.table, plan.coeffs(alphas, True),
                                                             div, n, int(rule), P, sh))
            plan.complete(sh)
            return plan.unpack()
        with torch.cuda.stream(st):
            host = self._cached("h_in64", (n + 1) * P, torch.float64, pinned=True)
            hv = host.numpy().reshape(n + 1, P)
            layout.pack(local, hv[0])
            for j, x in enumerate(nbrs):
                if callable(x):  # a filler writes the flat bucket itself (e.g. a payload decoder)
                    x(hv[j + 1])
                else:
                    layout.pack(x, hv[j + 1])
            dev = self._cached("d_in64", (n + 1) * P, torch.float64)
            dev.copy_(host, non_blocking=True)
            d = dev.view(n + 1, P)
            out = self._cached("d_out64", P, torch.float64)
            self.engine.fold_f64(out, d[0], [d[j] for j in range(1, n + 1)], [float(a) for a in alphas], rule,
                                 None if divisors is None else [float(x) for x in divisors], stream=st)
            h_out = self._cached("h_out64", P, torch.float64, pinned=True)
            h_out.copy_(out, non_blocking=True)
            st.synchronize()
            flat = h_out.numpy().copy()
        return layout.unpack(flat, copy=False)

    def mewma_tf1(self, W: Sequence, states: Sequence[np.ndarray], grads: Sequence[Sequence], rho: float,
                  lrs: Sequence[float], init: bool, use_filtered: bool) -> List[np.ndarray]:
        """CFA-GE update with the reference's fp64 operations (``cfa_mewma_tf1_f64``): ``W``
        (per-layer arrays), the neighbours' slot gradients ``grads[j]``, the caller's saved-state
        arrays ``states[k]`` [..., N] updated IN PLACE at slot j in their own dtype. Every
        operation is promoted as numpy 2 promotes it for the arrays' dtypes (Python-float rho and
        learning rates), so the result is the reference's: fp64 model arrays for its fp64
        gradients. ``lrs`` as in ``mewma``."""
        layout = _layout_of(W)
        n = len(grads)
        first_other = next((k for k in range(len(lrs)) if lrs[k] != lrs[0]), len(lrs))
        if any(lr != lrs[-1] for lr in lrs[first_other:]):
            raise ValueError("learning rates must be one value for the leading layers, one for the rest")
        split = int(layout.offsets[first_other])
        lr1, lr2 = float(lrs[0]), float(lrs[-1])
        from ..engine import TF1_GRAD_F32, TF1_STATE_F32, TF1_W_F32
        f32 = lambda a: _dtype(a) == _F32
        gf = [[f32(g[k]) for g in grads] for k in range(len(W))]
        flags = [(TF1_STATE_F32 if f32(states[k]) else 0) | (TF1_W_F32 if f32(W[k]) else 0)
                 | (TF1_GRAD_F32 if n and all(gf[k]) else 0) for k in range(len(W))]
        if n and any(len(set(gf[k])) > 1 for k in range(len(W))):
            raise ValueError("neighbour gradients of one layer must share a dtype")
        st_ = self._stream()
        if TF1_ZERO_COPY and n > 0:
            W_out = self._mewma_tf1_zero_copy(layout, W, states, grads, rho, lr1, lr2, split, init, use_filtered,
                                              flags, st_)
            u32 = lambda k: bool(flags[k] & (TF1_STATE_F32 if use_filtered else TF1_GRAD_F32))
            return [w.astype(np.float32) if (flags[k] & TF1_W_F32 and u32(k)) and f32(W[k]) else w
                    for k, w in enumerate(W_out)]
        with torch.cuda.stream(st_):
            dW = self._upload64(layout, W)
            ds = [self._upload64(layout, [np.asarray(st)[..., j] for st in states]) for j in range(n)]
            dg = [self._upload64(layout, g) for g in grads]
            for k0, k1, mask in self._runs(flags):
                b, e = layout.segment(k0)[0], layout.segment(k1 - 1)[1]
                self.engine.mewma_tf1_f64(dW[b:e], [x[b:e] for x in ds], [x[b:e] for x in dg], rho, lr1, lr2,
                                          max(0, min(split, e) - b), init, use_filtered, mask, stream=st_)
            W_out = dW.cpu().numpy()
            s_out = [x.cpu().numpy() for x in ds]
        for j in range(n):
            for k, arr in enumerate(layout.unpack(s_out[j], copy=False)):
                states[k][..., j] = arr
        # a model tensor stays fp32 only while every update it receives is fp32 (or none comes)
        u32 = lambda k: bool(flags[k] & (TF1_STATE_F32 if use_filtered else TF1_GRAD_F32))
        return [w.astype(np.float32) if (n == 0 or (flags[k] & TF1_W_F32 and u32(k))) and f32(W[k]) else w
                for k, w in enumerate(layout.unpack(W_out, copy=False))]


class _ZeroCopyPlan:
    """Reusable zero-copy state of one layout and fan-in on one thread (see HostMixer._zc_plan).

    Rows of ``pitch`` elements (16-byte multiples) in one pinned buffer: row 0 the local model,
    rows 1..n the neighbours; the output is a separate pinned row. The kernel reads and writes
    them through their device addresses over PCIe. ``views[m][k]`` is layer k of row m (flat),
    so a pack is one ``np.copyto`` per layer, with the same dtype conversion as
    ``BucketLayout.pack``."""

    def __init__(self, mixer: "HostMixer", layout: BucketLayout, n: int, dtype, out_dtype=None,
                 counter: bool = True):
        self.layout = layout
        shapes = layout.shapes
        self.P, self.n = self.layout.P, n
        self.dtype = np.dtype(dtype)
        align = 16 // self.dtype.itemsize
        self.pitch = self.P + (-self.P) % align
        tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64}
        self.host = torch.empty(max((n + 1) * self.pitch, 1), dtype=tdt[self.dtype], pin_memory=True)
        self.out = torch.empty(max(self.P, 1), dtype=tdt[np.dtype(out_dtype or dtype)], pin_memory=True)
        hv = self.host.numpy()[:(n + 1) * self.pitch].reshape(n + 1, self.pitch)
        self.rows = hv
        segs = [self.layout.segment(k) for k in range(len(shapes))]
        self.views = [[hv[m, b:e] for b, e in segs] for m in range(n + 1)]
        self.shaped_views = [[v.reshape(shp) for v, shp in zip(row, self.layout.shapes)] for row in self.views]
        self.out_np = self.out.numpy()[:self.P]
        self.out_slices = [(slice(b, e), shp) for (b, e), shp in zip(segs, self.layout.shapes)]
        eng = mixer.engine
        self.hb, self.ob = eng.host_device_ptr(self.host), eng.host_device_ptr(self.out)
        isz = self.dtype.itemsize
        self.table = _lib.ptr_table([self.hb + isz * self.pitch * (j + 1) for j in range(n)])
        self.lib = _lib.load()
        # completion word (cfa_stream_signal / cfa_wait_signal): one pinned 32-bit word per plan,
        # i.e. per thread and layout, set by the GPU to the call's sequence number
        self.sig_t = torch.zeros(16, dtype=torch.int32, pin_memory=True)
        self.sig_host, self.sig_dev = self.sig_t.data_ptr(), eng.host_device_ptr(self.sig_t)
        self.seq = 0
        self._coeffs = {}
        self._tables = {}
        self._runs = {}
        self._sh = None
        # compression count: a device counter (kernel atomics), read back by one 8-byte copy
        # into a pinned word and re-zeroed in the same stream order (cfa_counter_fetch). Only
        # the plans whose kernels take an epilogue get one; it is zeroed once, synchronously.
        self.counter_t = self.counter = self.count_pinned = self.count_host = None
        if counter:
            self.counter_t = torch.zeros(1, dtype=torch.int64, device=eng.device)
            torch.cuda.current_stream(eng.device).synchronize()
            self.counter = self.counter_t.data_ptr()
            self.count_pinned = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self.count_host = self.count_pinned.numpy()

    def complete(self, sh: int) -> None:
        """Waits until the plan's work on stream ``sh`` is done. With ``SIGNAL_COMPLETION`` a
        one-lane kernel after the work stores this call's sequence number into the plan's pinned
        word and the host spins on it (``cfa_wait_signal``): 17.0 -> 13.5 us per C1 call against
        hipStreamSynchronize's wake-up (``tools/probe/flag_sync.py``,
        ``profiles/r03v_flag_sync.jsonl``). Without the word after ``SIGNAL_SPIN_US`` the wait
        falls back to hipStreamSynchronize, which also reports an error of the stream's work."""
        if not SIGNAL_COMPLETION:
            _lib.check("cfa_stream_synchronize", self.lib.cfa_stream_synchronize(sh))
            return
        self.seq = self.seq % 0xFFFFFFFF + 1
        _lib.check("cfa_stream_signal", self.lib.cfa_stream_signal(self.sig_dev, self.seq, sh))
        _lib.check("cfa_wait_signal", self.lib.cfa_wait_signal(self.sig_host, self.seq, sh, SIGNAL_SPIN_US))

    def stream_handle(self, st) -> int:
        if self._sh is None or self._sh[0] is not st:
            self._sh = (st, int(st.cuda_stream))
        return self._sh[1]

    def coeffs(self, alphas, f64: bool = False):
        key = (tuple(alphas), f64)
        arr = self._coeffs.get(key)
        if arr is None:
            if len(self._coeffs) >= 64:
                self._coeffs.clear()
            arr = self._coeffs[key] = (_lib.double_array([float(a) for a in alphas]) if f64
                                       else _lib.float_array(list(alphas)))
        return arr

    def runs(self, flags: tuple):
        """HostMixer._runs(flags), cached per flag pattern."""
        r = self._runs.get(flags)
        if r is None:
            r = self._runs[flags] = HostMixer._runs(list(flags))
        return r

    def run_table(self, b: int):
        """Neighbour pointer table of the element offset ``b`` (one launch per dtype run)."""
        t = self._tables.get(b)
        if t is None:
            isz = self.dtype.itemsize
            t = self._tables[b] = _lib.ptr_table([self.hb + isz * (self.pitch * (j + 1) + b)
                                                  for j in range(self.n)])
        return t

    def row_table(self, first: int, count: int, b: int):
        """Pointer table of rows first..first+count-1 at element offset ``b`` (cached)."""
        key = ("rows", first, count, b)
        t = self._tables.get(key)
        if t is None:
            isz = self.dtype.itemsize
            t = self._tables[key] = _lib.ptr_table([self.hb + isz * (self.pitch * r + b)
                                                    for r in range(first, first + count)])
        return t

    def strides_one(self):
        t = self._tables.get("ones")
        if t is None:
            t = self._tables["ones"] = _lib.int64_array([1] * max(1, self.n))
        return t

    def pack(self, local, nbrs, require=None) -> bool:
        """Copy every model into its row (converting dtypes). With ``require`` (a dtype), stop and
        return False at the first array of another dtype or at a filler; True when packed."""
        sizes, shapes = self.layout.sizes, self.layout.shapes
        shaped = self.shaped_views
        for m, model in enumerate((local, *nbrs)):
            if callable(model):  # a filler writes the flat bucket itself (e.g. a payload decoder)
                if require is not None:
                    return False
                model(self.rows[m, :self.P])
                continue
            if len(model) != len(sizes):
                raise ValueError(f"expected {len(sizes)} tensors, got {len(model)}")
            for k, a in enumerate(model):
                if type(a) is np.ndarray and a.shape == shapes[k]:  # the common case: no reshape
                    if require is not None and a.dtype != require:
                        return False
                    np.copyto(shaped[m][k], a, casting="unsafe")
                    continue
                a = np.asarray(a)
                if require is not None and a.dtype != require:
                    return False
                if a.size != sizes[k]:
                    raise ValueError(f"tensor {k} has {a.size} elements, layout expects {sizes[k]}")
                np.copyto(self.views[m][k], a.reshape(-1), casting="unsafe")
        return True

    def fetch_count(self, sh: int) -> None:
        """Stream-ordered: the device counter's value into ``count_host`` and the counter reset
        (cfa_counter_fetch); the value is valid after the stream synchronisation."""
        _lib.check("cfa_counter_fetch", self.lib.cfa_counter_fetch(self.counter, self.count_pinned.data_ptr(), sh))

    def reset_count(self) -> None:
        """After a failed call: the counter may hold a partial sum; zero it (synchronously)."""
        self.counter_t.zero_()
        torch.cuda.synchronize(self.counter_t.device)

    def unpack(self) -> List[np.ndarray]:
        flat = self.out_np.copy()  # the pinned row is reused by the next call
        return [flat[sl].reshape(shp) for sl, shp in self.out_slices]


_mixers = {}
_mlock = threading.Lock()


def mixer() -> HostMixer:
    """Process-wide HostMixer on the current GPU (created on first use)."""
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None
    with _mlock:
        m = _mixers.get(dev)
        if m is None:
            m = _mixers[dev] = HostMixer(dev)
    return m
