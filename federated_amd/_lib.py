"""ctypes binding of ``libcfa.so`` (the C-ABI declared in ``include/cfa_engine.h``).

This is the thin shim between the Python consensus surface and the HIP kernels. There is no
fallback: if the library is missing or cannot be loaded, every compute entry point raises.

The library links against ``libamdhip64.so.7``/``librccl.so.1`` by soname. PyTorch-ROCm ships
its own copies of those libraries; importing torch first makes the dynamic loader bind
libcfa to the very same HIP runtime torch uses (same soname => same loaded object), so device
pointers and hipStream_t handles from torch tensors/streams are valid in libcfa.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  -- must be loaded before libcfa (see module docstring)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.environ.get("CFA_LIB", os.path.join(LIB_DIR, "libcfa.so"))

CFA_OK = 0
CFA_E_INVALID = -1
CFA_E_HIP = -2
CFA_E_RCCL = -3
CFA_E_UNSUPPORTED = -4
CFA_E_TIMEOUT = -5

CFA_MAX_FANIN = 16
CFA_UNIQUE_ID_BYTES = 128

RULE_SEQUENTIAL = 0
RULE_LINEAR = 1
RULE_SEQUENTIAL_DIV = 2
RULE_ACCUMULATE = 3

COMPRESS_NONE = 0
COMPRESS_SPARSE = 1
COMPRESS_SPARSE_DPCM = 2
COMPRESS_SPARSE_DPCM_HI = 3
COMPRESS_SPARSE_HI = 4

_c_float_p = ctypes.POINTER(ctypes.c_float)
_c_void_p = ctypes.c_void_p
_c_size_t = ctypes.c_size_t
_c_int = ctypes.c_int
_c_int64_p = ctypes.POINTER(ctypes.c_int64)
_c_int_p = ctypes.POINTER(ctypes.c_int)
_PP = ctypes.POINTER(ctypes.c_void_p)  # float* const* (host table of device pointers)


class LaneOp(ctypes.Structure):
    """cfa_lane_op (include/cfa_engine.h): one operation of a host-lane pump round."""
    _fields_ = [("wait_word", ctypes.c_void_p), ("wait_value", ctypes.c_uint), ("signal_value", ctypes.c_uint),
                ("signal_word", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("src", ctypes.c_void_p),
                ("bytes", ctypes.c_size_t), ("event", ctypes.c_void_p), ("mark", ctypes.c_int)]

# name -> (restype, argtypes); mirrors include/cfa_engine.h one for one.
SIGNATURES = {
    "cfa_version": (_c_int, []),
    "cfa_last_error": (ctypes.c_char_p, []),
    "cfa_device_prepare": (_c_int, [_c_int]),
    "cfa_stream_synchronize": (_c_int, [_c_void_p]),
    "cfa_counter_fetch": (_c_int, [_c_void_p, _c_void_p, _c_void_p]),
    "cfa_stream_signal": (_c_int, [_c_void_p, ctypes.c_uint, _c_void_p]),
    "cfa_wait_signal": (_c_int, [_c_void_p, ctypes.c_uint, _c_void_p, ctypes.c_longlong]),
    "cfa_host_register": (_c_int, [_c_void_p, _c_size_t]),
    "cfa_host_unregister": (_c_int, [_c_void_p]),
    "cfa_host_wait_word": (_c_int, [_c_void_p, ctypes.c_uint, ctypes.c_longlong]),
    "cfa_lane_pump_create": (_c_int, [ctypes.POINTER(_c_void_p), _c_void_p, _c_int, _c_int]),
    "cfa_lane_pump_submit": (_c_int, [_c_void_p, _c_void_p, _c_int, ctypes.c_longlong]),
    "cfa_lane_pump_wait": (_c_int, [_c_void_p, _c_int, ctypes.c_longlong]),
    "cfa_lane_pump_destroy": (_c_int, [_c_void_p]),
    "cfa_memcpy_async": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p]),
    "cfa_mix_seq_f32": (_c_int, [_c_void_p, _c_void_p, _PP, _c_float_p, _c_int, _c_size_t, _c_void_p]),
    "cfa_mix_seq_ex_f32": (_c_int, [_c_void_p, _c_void_p, _PP, _c_float_p, _c_int, _c_size_t,
                                    _c_void_p, _c_void_p]),
    "cfa_mix_seq_div_f32": (_c_int, [_c_void_p, _c_void_p, _PP, _c_float_p, _c_float_p, _c_int,
                                     _c_size_t, _c_void_p]),
    "cfa_mix_f32": (_c_int, [_c_void_p, _c_void_p, _PP, _c_float_p, _c_int, _c_size_t, _c_void_p]),
    "cfa_mix_seq_compress_f32": (_c_int, [_c_void_p, _c_void_p, _PP, _c_float_p, _c_int, _c_size_t,
                                          _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p]),
    "cfa_mix_tf1_f32": (_c_int, [_c_void_p, _c_void_p, _PP, ctypes.POINTER(ctypes.c_double), _c_int,
                                 _c_size_t, _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p]),
    "cfa_mix_tf1_ex_f32": (_c_int, [_c_void_p, _c_void_p, _PP, ctypes.POINTER(ctypes.c_double), _c_int,
                                    _c_size_t, _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p, _c_void_p]),
    "cfa_mix_tf1_wide_f32": (_c_int, [_c_void_p, _c_void_p, _PP, ctypes.POINTER(ctypes.c_double), _c_int,
                                      _c_size_t, _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p]),
    "cfa_mix_tf1_f64": (_c_int, [_c_void_p, _c_void_p, _PP, ctypes.POINTER(ctypes.c_double), _c_int, _c_int,
                                 _c_size_t, _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p]),
    "cfa_fold_f64": (_c_int, [_c_void_p, _c_void_p, _PP, ctypes.POINTER(ctypes.c_double),
                              ctypes.POINTER(ctypes.c_double), _c_int, _c_int, _c_size_t, _c_void_p]),
    "cfa_mewma_tf1_f64": (_c_int, [_c_void_p, _PP, _PP, _c_int64_p, _c_int, ctypes.c_double, ctypes.c_double,
                                   ctypes.c_double, _c_size_t, _c_int, _c_int, _c_int, _c_size_t, _c_void_p]),
    "cfa_compress_epilogue_f32": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_size_t, _c_void_p,
                                           _c_void_p]),
    "cfa_mewma_update_f32": (_c_int, [_c_void_p, _PP, _PP, _c_int64_p, _c_int, ctypes.c_double,
                                      ctypes.c_float, ctypes.c_float, _c_size_t, _c_int, _c_int,
                                      _c_size_t, _c_void_p]),
    "cfa_mix_window_f32": (_c_int, [_PP, _PP, _c_float_p, _c_int, _c_int, _c_int, _c_size_t, _c_void_p]),
    "cfa_mix_ring_round_f32": (_c_int, [_c_void_p, _c_void_p, _c_size_t, _c_void_p, _c_int, _c_int, _c_int,
                                        _c_size_t, _c_void_p]),
    "cfa_mix_population_tf1_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_int,
                                            _c_size_t, _c_int, _c_size_t, _c_size_t, _c_void_p, _c_void_p]),
    "cfa_mix_population_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                        _c_int, _c_int, _c_size_t, _c_void_p]),
    "cfa_ge_grad_cnn_f32": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                     _c_void_p, _c_void_p, _c_int, _c_void_p]),
    "cfa_ge_grad_2nn_f32": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p, _c_void_p,
                                     _c_int, _c_void_p]),
    "cfa_ge_grad_splits": (_c_int, [_c_int, _c_int, _c_size_t]),
    "cfa_ge_grad_workspace_elems": (_c_size_t, [_c_int, _c_int, _c_size_t]),
    "cfa_ge_grad_cnn_rows_f32": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                                          _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_size_t,
                                          _c_int, _c_void_p]),
    "cfa_ge_grad_2nn_rows_f32": (_c_int, [_c_void_p, _c_void_p, _c_int, _c_int, _c_int, _c_int, _c_void_p,
                                          _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_int,
                                          _c_void_p]),
    "cfa_ge_population_step_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                            _c_void_p, _c_int, ctypes.c_double, ctypes.c_float, ctypes.c_float,
                                            _c_size_t, _c_int, _c_size_t, _c_void_p, _c_void_p, _c_int, _c_int,
                                            _c_void_p]),
    "cfa_rccl_version": (_c_int, [_c_int_p]),
    "cfa_comm_unique_id": (_c_int, [_c_void_p]),
    "cfa_comm_init": (_c_int, [ctypes.POINTER(_c_void_p), _c_int, _c_int, _c_void_p, _c_int]),
    "cfa_comm_destroy": (_c_int, [_c_void_p]),
    "cfa_halo_exchange_f32": (_c_int, [_c_void_p, _PP, _c_int_p, _c_int, _PP, _c_int_p, _c_int,
                                       _c_size_t, _c_void_p]),
    "cfa_p2p_group_f32": (_c_int, [_c_void_p, _PP, ctypes.POINTER(_c_size_t), _c_int_p, _c_int, _PP,
                                   ctypes.POINTER(_c_size_t), _c_int_p, _c_int, _c_void_p]),
    "cfa_allreduce_sum_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_void_p]),
    "cfa_reduce_sum_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_size_t, _c_int, _c_void_p]),
    "cfa_mat_read": (_c_int, [ctypes.c_char_p, ctypes.POINTER(_c_void_p)]),
    "cfa_mat_free": (None, [_c_void_p]),
    "cfa_mat_num_vars": (_c_int, [_c_void_p]),
    "cfa_mat_vars": (_c_void_p, [_c_void_p]),
    "cfa_mat_header": (ctypes.c_char_p, [_c_void_p]),
    "cfa_mat_write": (_c_int, [ctypes.c_char_p, ctypes.c_char_p, _c_int, _c_void_p]),
    "cfa_host_mix_staging_elems": (_c_size_t, [_c_void_p, _c_int, _c_int, _c_size_t]),
    "cfa_host_mix_f32": (_c_int, [_c_void_p, _c_void_p, _c_void_p, _c_int, _c_int, _c_void_p, _c_void_p,
                                  _c_void_p, _c_size_t, _c_void_p, _c_size_t, _c_int, _c_void_p]),
    "cfa_npy_read": (_c_int, [ctypes.c_char_p, ctypes.POINTER(_c_void_p)]),
    "cfa_npy_parse": (_c_int, [_c_void_p, _c_size_t, ctypes.POINTER(_c_void_p)]),
    "cfa_npy_free": (None, [_c_void_p]),
    "cfa_npy_kind": (_c_int, [_c_void_p]),
    "cfa_npy_num_arrays": (_c_int, [_c_void_p]),
    "cfa_npy_arrays": (_c_void_p, [_c_void_p]),
    "cfa_payload_parse": (_c_int, [_c_void_p, _c_size_t, ctypes.POINTER(_c_void_p)]),
    "cfa_payload_free": (None, [_c_void_p]),
    "cfa_host_device_pointer": (_c_int, [_c_void_p, _PP]),
    "cfa_payload_num_keys": (_c_int, [_c_void_p]),
    "cfa_payload_key": (_c_int, [_c_void_p, _c_int, ctypes.POINTER(_c_void_p), ctypes.POINTER(_c_size_t)]),
    "cfa_payload_info": (_c_int, [_c_void_p, ctypes.c_char_p, _c_int_p, _c_int_p, _c_int64_p, _c_int64_p]),
    "cfa_payload_scalar": (_c_int, [_c_void_p, ctypes.c_char_p, _c_int_p, _c_int64_p,
                                    ctypes.POINTER(ctypes.c_double)]),
    "cfa_payload_read_f64": (_c_int, [_c_void_p, ctypes.c_char_p, _c_void_p, ctypes.c_int64]),
    "cfa_payload_read_f32": (_c_int, [_c_void_p, ctypes.c_char_p, _c_void_p, ctypes.c_int64]),
    "cfa_payload_encode": (_c_int, [_c_void_p, _c_int, _c_int, _c_void_p, _c_size_t,
                                    ctypes.POINTER(_c_size_t)]),
}

CFA_PAYLOAD_MAX_DIM = 8
PAYLOAD_NONE, PAYLOAD_BOOL, PAYLOAD_INT, PAYLOAD_FLOAT = 0, 1, 2, 3
PAYLOAD_F32_ARRAY, PAYLOAD_F64_ARRAY, PAYLOAD_I64_ARRAY, PAYLOAD_BOOL_ARRAY = 4, 5, 6, 7
PAYLOAD_STR, PAYLOAD_DICT = 8, 9


class PayloadItem(ctypes.Structure):
    """cfa_payload_item_t"""
    _fields_ = [("key", ctypes.c_char_p), ("kind", ctypes.c_int), ("data", ctypes.c_void_p),
                ("ndim", ctypes.c_int), ("shape", _c_int64_p), ("ivalue", ctypes.c_int64),
                ("fvalue", ctypes.c_double)]

class Launch(ctypes.Structure):
    """cfa_launch_t"""
    _fields_ = [("blocks_per_cu", ctypes.c_int), ("vec_per_lane", ctypes.c_int),
                ("nontemporal", ctypes.c_int)]


_lock = threading.Lock()
_lib = None


class CFAError(RuntimeError):
    """A libcfa call returned a negative status."""

    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed with code {code}: {msg}")
        self.code = code


def load() -> ctypes.CDLL:
    """Load libcfa.so once (thread-safe) and bind every C-ABI signature. Raises if missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.isfile(LIB_PATH):
                raise ImportError(
                    f"libcfa.so not found at {LIB_PATH}; build it with "
                    "`make -C federated_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`")
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


EXP_PATH = os.path.join(LIB_DIR, "libcfa_exp.so")
_exp = None


def load_experiments() -> ctypes.CDLL:
    """The measurement-only library of tools/ (tools/experiments/cfa_experiments.hip); never used by the
    product. Its entry points are bound by the tools themselves; errors via cfa_exp_last_error."""
    global _exp
    load()  # the HIP runtime torch loaded, as for libcfa
    with _lock:
        if _exp is None:
            if not os.path.isfile(EXP_PATH):
                raise ImportError(f"{EXP_PATH} not found; build it with `make -C federated_amd/csrc exp` "
                                  "(not part of the product build)")
            _exp = ctypes.CDLL(EXP_PATH, mode=ctypes.RTLD_LOCAL)
            _exp.cfa_exp_last_error.restype = ctypes.c_char_p
    return _exp


def call(name: str, *args) -> None:
    """Invoke a C-ABI entry point; raise CFAError with the library's message on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != CFA_OK:
        msg = lib.cfa_last_error()
        raise CFAError(name, rc, msg.decode() if msg else "")


def check(name: str, rc: int) -> None:
    """Raise CFAError for a non-zero status returned by a direct (pre-bound) entry-point call."""
    if rc != CFA_OK:
        msg = load().cfa_last_error()
        raise CFAError(name, rc, msg.decode() if msg else "")


def ptr_table(ptrs) -> "ctypes.Array":
    """Host array of device pointers (ints) for the `float* const*` arguments."""
    arr = (ctypes.c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def float_array(vals) -> "ctypes.Array":
    arr = (ctypes.c_float * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v
    return arr


def double_array(vals) -> "ctypes.Array":
    arr = (ctypes.c_double * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v
    return arr


def int64_array(vals) -> "ctypes.Array":
    arr = (ctypes.c_int64 * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v
    return arr


def size_array(vals) -> "ctypes.Array":
    arr = (ctypes.c_size_t * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v
    return arr


def int_array(vals) -> "ctypes.Array":
    arr = (ctypes.c_int * max(1, len(vals)))()
    for i, v in enumerate(vals):
        arr[i] = v
    return arr


def loaded_hip_runtimes() -> list:
    """Paths of every libamdhip64 mapped into this process (must be exactly one)."""
    paths = set()
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                if "libamdhip64" in line:
                    paths.add(line.split()[-1])
    except OSError:
        pass
    return sorted(paths)
