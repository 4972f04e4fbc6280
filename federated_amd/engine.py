"""Device-level consensus engine: the libcfa kernels on PyTorch-ROCm tensors.

PyTorch provides device memory and streams only; all arithmetic runs in the HIP kernels of
``libcfa.so`` (``federated_amd/csrc/cfa_*.hip``). Every call is asynchronous on the
given stream (default: torch's current stream on the tensor's device).

A *bucket* is a 1-D contiguous fp32 CUDA tensor holding one model (or gradient) flattened
layer by layer in the order the reference passes its tensors; ``BucketLayout`` maps the
reference's per-layer arrays to and from that flat form.
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
from typing import Iterable, Optional, Sequence

import numpy as np
import torch

from . import _lib

__all__ = ["Engine", "BucketLayout", "get_engine"]


def _require_gpu(device: Optional[torch.device]) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("federated_amd: no ROCm GPU visible; the consensus engine runs only on "
                           "MI355X (gfx950) through libcfa.so and has no CPU fallback")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise ValueError(f"engine device must be a cuda device, got {device}")
    return torch.device("cuda", device.index if device.index is not None else torch.cuda.current_device())


def _check_bucket(t: torch.Tensor, name: str, P: Optional[int] = None, dtype=torch.float32) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must live on the GPU (got {t.device})")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    n = t.numel()
    if P is not None and n != P:
        raise ValueError(f"{name} has {n} elements, expected {P}")
    return n


def _foreign(objs, index: int):
    """The first CUDA tensor or stream in ``objs`` (tensors, streams, and lists / tuples of them)
    that is not on GPU ``index``, else None."""
    for a in objs:
        for t in (a if isinstance(a, (list, tuple)) else (a,)):
            if isinstance(t, torch.Tensor):
                if t.is_cuda and t.device.index != index:
                    return t.device
            elif isinstance(t, torch.cuda.Stream) and t.device.index != index:
                return t.device
    return None


def _same_device(fn):
    """Engine method guard: every CUDA tensor and stream argument must be on the engine's GPU. A
    kernel enqueued on this GPU's stream with another GPU's pointers would fault (no peer mapping)
    or, with one, silently run over xGMI; both are caller errors, refused before any launch."""
    @functools.wraps(fn)
    def checked(self, *args, **kwargs):
        dev = _foreign(list(args) + list(kwargs.values()), self.device.index)
        if dev is not None:
            raise ValueError(f"{fn.__name__}: argument on {dev}, but this engine runs on {self.device}")
        return fn(self, *args, **kwargs)
    return checked


def _check_2d(t: torch.Tensor, name: str):
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.float32 or t.dim() != 2 \
            or not t.is_contiguous():
        raise TypeError(f"{name} must be a contiguous 2-D fp32 CUDA tensor")
    return int(t.shape[0]), int(t.shape[1])


TF1_STATE_F32, TF1_GRAD_F32, TF1_W_F32 = 1, 2, 4  # cfa_mewma_tf1_f64 dtype mask


class BucketLayout:
    """Offsets of a list of tensors flattened into one bucket (layer order preserved)."""

    def __init__(self, shapes: Iterable[Sequence[int]]):
        self.shapes = [tuple(int(d) for d in s) for s in shapes]
        self.sizes = [int(np.prod(s)) if len(s) else 1 for s in self.shapes]
        self.offsets = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        self.P = int(self.offsets[-1])

    @classmethod
    def of(cls, arrays) -> "BucketLayout":
        return cls([np.shape(a) for a in arrays])

    def segment(self, k: int) -> tuple:
        return int(self.offsets[k]), int(self.offsets[k + 1])

    def pack(self, arrays, out: Optional[np.ndarray] = None) -> np.ndarray:
        """Flatten per-layer arrays into ``out`` (length P; fp32 unless ``out`` says otherwise),
        converting dtype if needed."""
        if out is None:
            out = np.empty(self.P, dtype=np.float32)
        if len(arrays) != len(self.sizes):
            raise ValueError(f"expected {len(self.sizes)} tensors, got {len(arrays)}")
        for k, a in enumerate(arrays):
            a = np.asarray(a)
            if a.size != self.sizes[k]:
                raise ValueError(f"tensor {k} has {a.size} elements, layout expects {self.sizes[k]}")
            b, e = self.segment(k)
            out[b:e] = a.reshape(-1)
        return out

    def unpack(self, flat: np.ndarray, copy: bool = True) -> list:
        res = []
        for k, shp in enumerate(self.shapes):
            b, e = self.segment(k)
            v = flat[b:e].reshape(shp)
            res.append(v.copy() if copy else v)
        return res


class Engine:
    """libcfa kernels bound to one GPU."""

    def __init__(self, device=None):
        self.device = _require_gpu(device)
        self.lib = _lib.load()
        # device attributes cached and kernel LDS limits raised now, so no launch queries the
        # device (hipGraph captures of engine launches run in the strict mode)
        _lib.call("cfa_device_prepare", int(self.device.index))

    # -- helpers ---------------------------------------------------------------------------
    def stream_handle(self, stream: Optional[torch.cuda.Stream] = None) -> int:
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return int(s.cuda_stream)

    def empty(self, P: int) -> torch.Tensor:
        return torch.empty(P, dtype=torch.float32, device=self.device)

    def counter(self) -> torch.Tensor:
        return torch.zeros(1, dtype=torch.int64, device=self.device)

    # -- mixing ----------------------------------------------------------------------------
    def mix_seq(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                alphas: Sequence[float], stream=None, launch: Optional[tuple] = None) -> torch.Tensor:
        """out = fold_j(w <- w + alphas[j]*(nbrs[j] - w)), w0 = local (sequential CFA rule).
        ``launch`` = (blocks_per_cu, vec_per_lane, nontemporal) overrides the launch shape."""
        P = _check_bucket(local, "local")
        _check_bucket(out, "out", P)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P)
        if len(alphas) != len(nbrs):
            raise ValueError("one alpha per neighbour required")
        table = _lib.ptr_table([x.data_ptr() for x in nbrs])
        if launch is None:
            _lib.call("cfa_mix_seq_f32", out.data_ptr(), local.data_ptr(), table,
                      _lib.float_array(alphas), len(nbrs), P, self.stream_handle(stream))
        else:
            lc = _lib.Launch(*launch)
            _lib.call("cfa_mix_seq_ex_f32", out.data_ptr(), local.data_ptr(), table,
                      _lib.float_array(alphas), len(nbrs), P, ctypes.addressof(lc),
                      self.stream_handle(stream))
        return out

    def prepare_mix_seq(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                        alphas: Sequence[float]):
        """mix_seq with its checks and ctypes tables done once: returns ``launch(stream=None)``,
        which enqueues the same kernel with one foreign call. For rounds that repeat the same
        mixes on resident buffers (population shards), where per-launch Python work would
        otherwise approach the kernel time at small buckets. The tensors must stay alive."""
        P = _check_bucket(local, "local")
        _check_bucket(out, "out", P)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P)
        if len(alphas) != len(nbrs):
            raise ValueError("one alpha per neighbour required")
        table = _lib.ptr_table([x.data_ptr() for x in nbrs])
        coeff = _lib.float_array(alphas)
        fn = self.lib.cfa_mix_seq_f32
        args = (out.data_ptr(), local.data_ptr(), table, coeff, len(nbrs), P)
        keep = (out, local, tuple(nbrs), table, coeff)
        dev = self.device

        def launch(stream=None):
            s = stream if stream is not None else torch.cuda.current_stream(dev)
            rc = fn(*args, s.cuda_stream)
            if rc != _lib.CFA_OK:
                msg = self.lib.cfa_last_error()
                raise _lib.CFAError("cfa_mix_seq_f32", rc, msg.decode() if msg else "")

        launch.keep = keep
        return launch

    @staticmethod
    def host_device_ptr(t: torch.Tensor) -> int:
        """Device address of a pinned host tensor (cfa_host_device_pointer)."""
        if not isinstance(t, torch.Tensor) or t.is_cuda or not t.is_pinned():
            raise ValueError("expected a pinned host tensor (pin_memory=True)")
        if not t.is_contiguous():
            raise TypeError("expected a contiguous tensor")
        dev = ctypes.c_void_p()
        _lib.call("cfa_host_device_pointer", ctypes.c_void_p(t.data_ptr()), ctypes.byref(dev))
        return int(dev.value)

    def mix_seq_pinned(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                       alphas: Sequence[float], stream=None) -> torch.Tensor:
        """mix_seq on buckets that live in pinned HOST memory (f2): the kernel reads them over
        PCIe and writes ``out`` (pinned host) directly, with no staging copies, so the link's
        read and write directions overlap. Asynchronous on ``stream`` like mix_seq; the caller
        synchronises before reading ``out``. Results equal mix_seq on device copies."""
        P = local.numel()
        for name, t in [("out", out), ("local", local)] + [(f"nbrs[{j}]", x) for j, x in enumerate(nbrs)]:
            if t.dtype != torch.float32:
                raise TypeError(f"{name} must be fp32 (got {t.dtype})")
            if t.numel() != P:
                raise ValueError(f"{name} has {t.numel()} elements, expected {P}")
        if len(alphas) != len(nbrs):
            raise ValueError("one alpha per neighbour required")
        table = _lib.ptr_table([self.host_device_ptr(x) for x in nbrs])
        _lib.call("cfa_mix_seq_f32", self.host_device_ptr(out), self.host_device_ptr(local), table,
                  _lib.float_array(alphas), len(nbrs), P, self.stream_handle(stream))
        return out

    def mix_seq_div(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                    alphas: Sequence[float], divisors: Sequence[float], stream=None) -> torch.Tensor:
        """out = fold_j(w <- w + (alphas[j]*(nbrs[j] - w)) / divisors[j]) (FedAvg form)."""
        P = _check_bucket(local, "local")
        _check_bucket(out, "out", P)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P)
        if not (len(alphas) == len(divisors) == len(nbrs)):
            raise ValueError("one alpha and one divisor per neighbour required")
        _lib.call("cfa_mix_seq_div_f32", out.data_ptr(), local.data_ptr(),
                  _lib.ptr_table([x.data_ptr() for x in nbrs]), _lib.float_array(alphas),
                  _lib.float_array(divisors), len(nbrs), P, self.stream_handle(stream))
        return out

    def mix_linear(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                   coeff: Sequence[float], stream=None) -> torch.Tensor:
        """out = coeff[0]*local + sum_j coeff[j+1]*nbrs[j]."""
        P = _check_bucket(local, "local")
        _check_bucket(out, "out", P)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P)
        if len(coeff) != len(nbrs) + 1:
            raise ValueError("len(coeff) must be len(nbrs) + 1")
        _lib.call("cfa_mix_f32", out.data_ptr(), local.data_ptr(),
                  _lib.ptr_table([x.data_ptr() for x in nbrs]), _lib.float_array(coeff),
                  len(nbrs), P, self.stream_handle(stream))
        return out

    def mix_seq_compress(self, out: torch.Tensor, local: torch.Tensor,
                         nbrs: Sequence[torch.Tensor], alphas: Sequence[float], mode: int,
                         cbegin: int, cend: int, kept: torch.Tensor, stream=None) -> torch.Tensor:
        """Sequential mix fused with the cfa_ongraphs compression epilogue on [cbegin, cend).
        Adds the kept-parameter count to ``kept`` (int64 CUDA tensor of one element)."""
        P = _check_bucket(local, "local")
        _check_bucket(out, "out", P)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P)
        self._check_counter(kept)
        if len(alphas) != len(nbrs):
            raise ValueError("one alpha per neighbour required")
        _lib.call("cfa_mix_seq_compress_f32", out.data_ptr(), local.data_ptr(),
                  _lib.ptr_table([x.data_ptr() for x in nbrs]), _lib.float_array(alphas),
                  len(nbrs), P, int(mode), int(cbegin), int(cend), kept.data_ptr(),
                  self.stream_handle(stream))
        return out

    def mix_tf1(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                alphas: Sequence[float], mode: int = 0, cbegin: int = 0, cend: int = 0,
                kept: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """TF1 mix with the reference's numpy-2 numerics (fp32 first subtraction, fp64 chain,
        fp64 compression epilogue on [cbegin, cend), one rounding to fp32). ``alphas`` are the
        float64 products eps * wf_j. ``kept`` (int64 CUDA tensor of one element) is required
        when ``mode`` != 0."""
        P = _check_bucket(local, "local")
        _check_bucket(out, "out", P)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P)
        if kept is not None:
            self._check_counter(kept)
        if len(alphas) != len(nbrs):
            raise ValueError("one alpha per neighbour required")
        # above CFA_MAX_FANIN the passes chain through an fp64 scratch bucket from torch's
        # allocator (stream-ordered, and capturable), not a library allocation. It is allocated
        # on the stream the kernel writes it on: a block from another stream's pool could still
        # be in use by work queued there.
        scratch = None
        if len(nbrs) > _lib.CFA_MAX_FANIN:
            ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
            with ctx:
                scratch = torch.empty(P, dtype=torch.float64, device=self.device)
        _lib.call("cfa_mix_tf1_ex_f32", out.data_ptr(), local.data_ptr(),
                  _lib.ptr_table([x.data_ptr() for x in nbrs]), _lib.double_array(alphas),
                  len(nbrs), P, int(mode), int(cbegin), int(cend),
                  kept.data_ptr() if kept is not None else None,
                  scratch.data_ptr() if scratch is not None else None, self.stream_handle(stream))
        return out

    def mix_tf1_f64(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                    alphas: Sequence[float], step0_f32: bool, mode: int = 0, cbegin: int = 0,
                    cend: int = 0, kept: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """TF1 mix on fp64 buckets (cfa_mix_tf1_f64): the reference's fp64 chain, unrounded.
        ``step0_f32``: the reference's local and first-neighbour arrays are both fp32."""
        F64 = torch.float64
        P = _check_bucket(local, "local", dtype=F64)
        _check_bucket(out, "out", P, F64)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P, F64)
        if kept is not None:
            self._check_counter(kept)
        if len(alphas) != len(nbrs):
            raise ValueError("one alpha per neighbour required")
        _lib.call("cfa_mix_tf1_f64", out.data_ptr(), local.data_ptr(),
                  _lib.ptr_table([x.data_ptr() for x in nbrs]), _lib.double_array(alphas), len(nbrs),
                  int(bool(step0_f32)), P, int(mode), int(cbegin), int(cend),
                  kept.data_ptr() if kept is not None else None, self.stream_handle(stream))
        return out

    def fold_f64(self, out: torch.Tensor, local: torch.Tensor, nbrs: Sequence[torch.Tensor],
                 alphas: Sequence[float], rule: int, divisors: Optional[Sequence[float]] = None,
                 stream=None) -> torch.Tensor:
        """fp64 fold (cfa_fold_f64): SEQUENTIAL, SEQUENTIAL_DIV (``divisors``) or ACCUMULATE."""
        F64 = torch.float64
        P = _check_bucket(local, "local", dtype=F64)
        _check_bucket(out, "out", P, F64)
        for j, x in enumerate(nbrs):
            _check_bucket(x, f"nbrs[{j}]", P, F64)
        if len(alphas) != len(nbrs) or (divisors is not None and len(divisors) != len(nbrs)):
            raise ValueError("one alpha (and one divisor, when given) per neighbour required")
        _lib.call("cfa_fold_f64", out.data_ptr(), local.data_ptr(),
                  _lib.ptr_table([x.data_ptr() for x in nbrs]), _lib.double_array(alphas),
                  _lib.double_array(divisors) if divisors is not None else None, len(nbrs), int(rule), P,
                  self.stream_handle(stream))
        return out

    def mewma_tf1_f64(self, W: torch.Tensor, s: Sequence[torch.Tensor], g: Sequence[torch.Tensor],
                      rho: float, lr1: float, lr2: float, lr_split: int, init: bool,
                      use_filtered: bool, f32_mask: int = 0, stream=None) -> torch.Tensor:
        """CFA-GE MEWMA on fp64 buckets (cfa_mewma_tf1_f64); W and s_j in place. ``g`` may be
        element-strided 1-D fp64 views. ``f32_mask``: which reference arrays are fp32
        (TF1_STATE_F32 | TF1_GRAD_F32 | TF1_W_F32)."""
        F64 = torch.float64
        P = _check_bucket(W, "W", dtype=F64)
        if len(s) != len(g):
            raise ValueError("one state bucket per gradient bucket")
        strides = []
        for j in range(len(g)):
            _check_bucket(s[j], f"s[{j}]", P, F64)
            gj = g[j]
            if not gj.is_cuda or gj.dtype != F64 or gj.dim() != 1 or gj.numel() != P:
                raise ValueError(f"g[{j}] must be a 1-D fp64 CUDA view of {P} elements")
            strides.append(int(gj.stride(0)))
        _lib.call("cfa_mewma_tf1_f64", W.data_ptr(), _lib.ptr_table([x.data_ptr() for x in s]),
                  _lib.ptr_table([x.data_ptr() for x in g]), _lib.int64_array(strides), len(g),
                  float(rho), float(lr1), float(lr2), int(lr_split), int(bool(init)),
                  int(bool(use_filtered)), int(f32_mask), P, self.stream_handle(stream))
        return W

    def compress(self, y: torch.Tensor, ref: Optional[torch.Tensor], mode: int,
                 kept: torch.Tensor, stream=None) -> torch.Tensor:
        P = _check_bucket(y, "y")
        if ref is not None:
            _check_bucket(ref, "ref", P)
        self._check_counter(kept)
        _lib.call("cfa_compress_epilogue_f32", y.data_ptr(), ref.data_ptr() if ref is not None else None,
                  int(mode), P, kept.data_ptr(), self.stream_handle(stream))
        return y

    @staticmethod
    def _check_counter(kept: torch.Tensor) -> None:
        if not (isinstance(kept, torch.Tensor) and kept.is_cuda and kept.dtype == torch.int64
                and kept.numel() >= 1):
            raise TypeError("kept must be an int64 CUDA tensor")

    # -- CFA-GE ----------------------------------------------------------------------------
    def mewma(self, W: torch.Tensor, s: Sequence[torch.Tensor], g: Sequence[torch.Tensor],
              rho: float, lr1: float, lr2: float, lr_split: int, init: bool, use_filtered: bool,
              stream=None) -> torch.Tensor:
        """CFA-GE update: for each j, s_j <- init ? g_j : rho*g_j + (1-rho)*s_j;
        W <- W - lr*(use_filtered ? s_j : g_j) with lr = lr1 below lr_split, lr2 above."""
        P = _check_bucket(W, "W")
        if len(s) != len(g):
            raise ValueError("one state bucket per gradient bucket")
        strides = []
        for j in range(len(g)):
            _check_bucket(s[j], f"s[{j}]", P)
            gj = g[j]
            if not gj.is_cuda or gj.dtype != torch.float32 or gj.dim() != 1 or gj.numel() != P:
                raise ValueError(f"g[{j}] must be a 1-D fp32 CUDA view of {P} elements")
            strides.append(int(gj.stride(0)))
        _lib.call("cfa_mewma_update_f32", W.data_ptr(), _lib.ptr_table([x.data_ptr() for x in s]),
                  _lib.ptr_table([x.data_ptr() for x in g]), _lib.int64_array(strides), len(g),
                  float(rho), float(lr1), float(lr2), int(lr_split), int(bool(init)),
                  int(bool(use_filtered)), P, self.stream_handle(stream))
        return W

    # -- CFA-GE neighbour gradients (f3) ---------------------------------------------------
    def _grad_args(self, x, y, models, grads):
        B, L = _check_2d(x, "x")
        By, C = _check_2d(y, "y")
        M, P = _check_2d(models, "models")
        if By != B:
            raise ValueError("x and y must hold the same number of samples")
        if tuple(grads.shape) != (M, P):
            raise ValueError("grads must have the shape of models")
        _check_2d(grads, "grads")
        return B, L, C, M, P

    def grad_cnn(self, x: torch.Tensor, y: torch.Tensor, models: torch.Tensor, grads: torch.Tensor,
                 filter: int, number: int, stride: int, stream=None) -> torch.Tensor:
        """Gradients of the CNN cost (cfa_ge_2stage.py:392-405, :425-430) at each row of
        ``models`` [M, P] (TF1 bucket order W1 b1 W2 b2) into ``grads`` [M, P]."""
        B, L, C, M, P = self._grad_args(x, y, models, grads)
        L2 = -(-(-(-L // stride)) // stride)
        if P != filter * number + number + L2 * number * C + C:
            raise ValueError(f"CNN bucket of {P} parameters does not match filter {filter}, number {number}, "
                             f"stride {stride}, {L} inputs, {C} classes (multip must be {L2})")
        _lib.call("cfa_ge_grad_cnn_f32", x.data_ptr(), y.data_ptr(), B, L, C, int(filter), int(number),
                  int(stride), models.data_ptr(), grads.data_ptr(), M, self.stream_handle(stream))
        return grads

    def grad_2nn(self, x: torch.Tensor, y: torch.Tensor, models: torch.Tensor, grads: torch.Tensor,
                 hidden: int, stream=None) -> torch.Tensor:
        """Gradients of the 2NN cost (cfa_ge_2stage.py:407-420, :425-430); see grad_cnn."""
        B, L, C, M, P = self._grad_args(x, y, models, grads)
        if P != L * hidden + hidden + hidden * C + C:
            raise ValueError(f"2NN bucket of {P} parameters does not match {L} inputs, {hidden} hidden, {C} classes")
        _lib.call("cfa_ge_grad_2nn_f32", x.data_ptr(), y.data_ptr(), B, L, int(hidden), C, models.data_ptr(),
                  grads.data_ptr(), M, self.stream_handle(stream))
        return grads

    def grad_workspace(self, M: int, B: int, P: int) -> torch.Tensor:
        """Workspace for the batch-split gradient launch (cfa_ge_grad_workspace_elems)."""
        n = int(_lib.load().cfa_ge_grad_workspace_elems(int(M), int(B), int(P)))
        return torch.empty(max(n, 1), dtype=torch.float32, device=self.device)

    def grad_splits(self, M: int, B: int, P: int) -> int:
        """Workgroups per evaluation of a split gradient launch (cfa_ge_grad_splits)."""
        return int(_lib.load().cfa_ge_grad_splits(int(M), int(B), int(P)))

    def grad_rows(self, ml_model: int, x: torch.Tensor, y: torch.Tensor, models: torch.Tensor,
                  model_row: torch.Tensor, data_row: torch.Tensor, grads: Optional[torch.Tensor], geom: dict,
                  stream=None, workspace: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """Population form (cfa_ge_grad_{cnn,2nn}_rows_f32): evaluation m = gradient of data row
        data_row[m] (x [Dx, B, L], y [Dx, B, C]) at model row model_row[m] of models [Dm, P],
        into grads [M, P]. ``geom``: filter/number/stride (CNN) or intermediate_nodes (2NN).
        ``workspace`` (``grad_workspace``) lets each evaluation's batch spread over workgroups.
        ``grads=None``: partials only, [M][grad_splits(M, B, P)][P] into ``workspace`` (at least
        that size), summed later by ``ge_population_step(..., reduce=...)``."""
        for name, t, nd in (("x", x, 3), ("y", y, 3)):
            if not t.is_cuda or t.dtype != torch.float32 or t.dim() != nd or not t.is_contiguous():
                raise TypeError(f"{name} must be a contiguous 3-D fp32 CUDA tensor")
        Dm, P = _check_2d(models, "models")
        if grads is None:
            if workspace is None:
                raise ValueError("a partials-only launch (grads=None) needs a workspace")
            M, Pg = int(model_row.numel()), P
            need = M * self.grad_splits(M, int(x.shape[1]), P) * P
            if workspace.numel() < need:
                raise ValueError(f"partials-only launch needs a workspace of {need} floats")
        else:
            M, Pg = _check_2d(grads, "grads")
        for name, t in (("model_row", model_row), ("data_row", data_row)):
            if not t.is_cuda or t.dtype != torch.int32 or t.numel() != M or not t.is_contiguous():
                raise TypeError(f"{name} must be a contiguous int32 CUDA tensor of {M} entries")
        Dx, B, L = (int(v) for v in x.shape)
        if tuple(y.shape[:2]) != (Dx, B) or Pg != P:
            raise ValueError("y must be [Dx, B, C] and grads [M, P]")
        C = int(y.shape[2])
        ws_ptr, ws_n = None, 0
        if workspace is not None:
            if not workspace.is_cuda or workspace.dtype != torch.float32 or not workspace.is_contiguous():
                raise TypeError("workspace must be a contiguous fp32 CUDA tensor")
            ws_ptr, ws_n = workspace.data_ptr(), workspace.numel()
        if ml_model == 1:
            F, NC, S = int(geom["filter"]), int(geom["number"]), int(geom["stride"])
            L2 = -(-(-(-L // S)) // S)
            if P != F * NC + NC + L2 * NC * C + C:
                raise ValueError("CNN bucket size does not match the geometry")
            _lib.call("cfa_ge_grad_cnn_rows_f32", x.data_ptr(), y.data_ptr(), B, L, C, F, NC, S, models.data_ptr(),
                      model_row.data_ptr(), data_row.data_ptr(), None if grads is None else grads.data_ptr(), ws_ptr,
                      ws_n, M, self.stream_handle(stream))
        elif ml_model == 2:
            H = int(geom["intermediate_nodes"])
            if P != L * H + H + H * C + C:
                raise ValueError("2NN bucket size does not match the geometry")
            _lib.call("cfa_ge_grad_2nn_rows_f32", x.data_ptr(), y.data_ptr(), B, L, H, C, models.data_ptr(),
                      model_row.data_ptr(), data_row.data_ptr(), None if grads is None else grads.data_ptr(), ws_ptr,
                      ws_n, M, self.stream_handle(stream))
        else:
            raise ValueError("ml_model must be 1 (CNN) or 2 (2NN)")
        return grads

    # -- population ------------------------------------------------------------------------
    def mix_window(self, outs: Sequence[torch.Tensor], rows: Sequence[torch.Tensor], alphas: Sequence[Sequence[float]],
                   hl: int, hr: int, stream=None) -> None:
        """One sliding-window pass (cfa_mix_window_f32): len(outs) consecutive devices, rows =
        the window's len(outs) + hl + hr buckets in device order, alphas[b] = device b's step
        coefficients (hl + hr values, all equal: the kernel takes one per device)."""
        nb = len(outs)
        if len(rows) != nb + hl + hr or len(alphas) != nb:
            raise ValueError("window needs nb + hl + hr rows and one alpha list per device")
        P = _check_bucket(rows[0], "rows[0]")
        for k, r in enumerate(rows):
            _check_bucket(r, f"rows[{k}]", P)
        for b, o in enumerate(outs):
            _check_bucket(o, f"outs[{b}]", P)
        per_dev = []
        for b, al in enumerate(alphas):
            al = [float(a) for a in al]
            if len(al) != hl + hr or len(set(al)) > 1:
                raise ValueError(f"device {b}: the window pass needs hl + hr equal alphas, got {al}")
            per_dev.append(al[0] if al else 0.0)
        _lib.call("cfa_mix_window_f32", _lib.ptr_table([o.data_ptr() for o in outs]),
                  _lib.ptr_table([r.data_ptr() for r in rows]), _lib.float_array(per_dev), nb, int(hl), int(hr), P,
                  self.stream_handle(stream))
    def ring_round(self, out: torch.Tensor, models: torch.Tensor, alphas: torch.Tensor, hl: int, hr: int,
                   stream=None) -> torch.Tensor:
        """cfa_mix_ring_round_f32: one launch mixing every device of a stacked [D, P] population
        with its ring window [d-hl .. d-1, d+1 .. d+hr] (mod D); ``alphas`` [D] fp32 CUDA (one
        coefficient per device); out [D, P] must not overlap models."""
        D, P = _check_2d(models, "models")
        if tuple(out.shape) != (D, P) or not out.is_cuda or out.dtype != torch.float32 or not out.is_contiguous():
            raise TypeError("out must be a contiguous [D, P] fp32 CUDA tensor")
        if not alphas.is_cuda or alphas.dtype != torch.float32 or alphas.numel() != D or not alphas.is_contiguous():
            raise TypeError("alphas must be a contiguous fp32 CUDA tensor of D entries")
        _lib.call("cfa_mix_ring_round_f32", out.data_ptr(), models.data_ptr(), P, alphas.data_ptr(), D, int(hl),
                  int(hr), P, self.stream_handle(stream))
        return out

    def ge_population_step(self, out_ptrs: torch.Tensor, src_ptrs: torch.Tensor, state_ptrs: torch.Tensor,
                           grad_ptrs: torch.Tensor, csr_ptr: torch.Tensor, csr_idx: torch.Tensor,
                           csr_coef: torch.Tensor, D: int, rho: float, lr1: float, lr2: float, lr_split: int,
                           use_filtered: bool, P: int, stream=None, reduce=None) -> None:
        """cfa_ge_population_step_f32: stage-1 mix + MEWMA gradient step of D devices in one
        launch; pointer tables are int64 CUDA tensors aligned with the CSR entries.
        ``reduce=(workspace, out [M, P], splits)``: the same launch also sums a partials-only
        gradient launch's [M][splits][P] workspace into ``out``."""
        for name, t, dt in (("out_ptrs", out_ptrs, torch.int64), ("src_ptrs", src_ptrs, torch.int64),
                            ("state_ptrs", state_ptrs, torch.int64), ("grad_ptrs", grad_ptrs, torch.int64),
                            ("csr_ptr", csr_ptr, torch.int32), ("csr_idx", csr_idx, torch.int32),
                            ("csr_coef", csr_coef, torch.float32)):
            if not t.is_cuda or t.dtype != dt or not t.is_contiguous():
                raise TypeError(f"{name} must be a contiguous {dt} CUDA tensor")
        E = csr_idx.numel()
        if csr_ptr.numel() != D + 1 or out_ptrs.numel() != D or state_ptrs.numel() != E or grad_ptrs.numel() != E:
            raise ValueError("tables: D+1 row pointers, D outputs, one state and one gradient slot per CSR entry")
        r_ws = r_out = None
        r_M = r_sp = 0
        if reduce is not None:
            ws, out, r_sp = reduce
            r_M, Po = _check_2d(out, "reduce out")
            r_sp = int(r_sp)
            if Po != P or r_sp < 1 or not ws.is_cuda or ws.dtype != torch.float32 or ws.numel() < r_M * r_sp * P:
                raise ValueError("reduce: out [M, P] and a workspace of M * splits * P fp32 elements")
            r_ws, r_out = ws.data_ptr(), out.data_ptr()
        _lib.call("cfa_ge_population_step_f32", out_ptrs.data_ptr(), src_ptrs.data_ptr(), state_ptrs.data_ptr(),
                  grad_ptrs.data_ptr(), csr_ptr.data_ptr(), csr_idx.data_ptr(), csr_coef.data_ptr(), int(D),
                  float(rho), float(lr1), float(lr2), int(lr_split), int(bool(use_filtered)), int(P), r_ws, r_out,
                  int(r_M), int(r_sp), self.stream_handle(stream))

    def population_tf1(self, out_ptrs: torch.Tensor, src_ptrs: torch.Tensor, csr_ptr: torch.Tensor,
                       csr_idx: torch.Tensor, csr_coef64: torch.Tensor, D: int, P: int, stream=None,
                       mode: int = 0, cbegin: int = 0, cend: int = 0,
                       kept: Optional[torch.Tensor] = None) -> None:
        """One launch mixing D devices with the TF1 numerics (cfa_mix_population_tf1_f32):
        fp32 first subtraction, fp64 chain with fp64 coefficients, one rounding to fp32.
        ``mode`` != 0: the compression epilogue on [cbegin, cend) of every device, counts added
        to ``kept`` (int64 CUDA tensor of D zeroed counters)."""
        for name, t, dt in (("out_ptrs", out_ptrs, torch.int64), ("src_ptrs", src_ptrs, torch.int64),
                            ("csr_ptr", csr_ptr, torch.int32), ("csr_idx", csr_idx, torch.int32),
                            ("csr_coef64", csr_coef64, torch.float64)):
            if not t.is_cuda or t.dtype != dt or not t.is_contiguous():
                raise TypeError(f"{name} must be a contiguous {dt} CUDA tensor")
        if csr_ptr.numel() != D + 1 or out_ptrs.numel() != D:
            raise ValueError("csr_ptr must have D+1 entries and out_ptrs D entries")
        if mode and (kept is None or not kept.is_cuda or kept.dtype != torch.int64 or kept.numel() != D):
            raise TypeError("compression needs kept: an int64 CUDA tensor of D counters")
        _lib.call("cfa_mix_population_tf1_f32", out_ptrs.data_ptr(), src_ptrs.data_ptr(), csr_ptr.data_ptr(),
                  csr_idx.data_ptr(), csr_coef64.data_ptr(), int(D), int(P), int(mode), int(cbegin), int(cend),
                  kept.data_ptr() if kept is not None else None, self.stream_handle(stream))

    def population(self, out_ptrs: torch.Tensor, src_ptrs: torch.Tensor, csr_ptr: torch.Tensor,
                   csr_idx: torch.Tensor, csr_coef: torch.Tensor, D: int, rule: int, P: int,
                   stream=None) -> None:
        """One launch mixing D devices; tables are device tensors (int64 pointers, int32 CSR,
        fp32 coefficients). See cfa_mix_population_f32."""
        for name, t, dt in (("out_ptrs", out_ptrs, torch.int64), ("src_ptrs", src_ptrs, torch.int64),
                            ("csr_ptr", csr_ptr, torch.int32), ("csr_idx", csr_idx, torch.int32),
                            ("csr_coef", csr_coef, torch.float32)):
            if not t.is_cuda or t.dtype != dt or not t.is_contiguous():
                raise TypeError(f"{name} must be a contiguous {dt} CUDA tensor")
        if csr_ptr.numel() != D + 1 or out_ptrs.numel() != D:
            raise ValueError("csr_ptr must have D+1 entries and out_ptrs D entries")
        _lib.call("cfa_mix_population_f32", out_ptrs.data_ptr(), src_ptrs.data_ptr(),
                  csr_ptr.data_ptr(), csr_idx.data_ptr(), csr_coef.data_ptr(), int(D), int(rule),
                  int(P), self.stream_handle(stream))


_engines: dict = {}


for _name, _fn in list(vars(Engine).items()):
    if (callable(_fn) and not isinstance(_fn, (staticmethod, classmethod)) and not _name.startswith("_")
            and _name not in ("empty", "counter", "stream_handle", "grad_workspace", "grad_splits")):
        setattr(Engine, _name, _same_device(_fn))


def get_engine(device=None) -> Engine:
    """Process-wide engine per device (the engine object itself holds no mutable state)."""
    dev = _require_gpu(device)
    eng = _engines.get(dev.index)
    if eng is None:
        eng = _engines[dev.index] = Engine(dev)
    return eng
