"""MATLAB level-5 files of the TF1 exchange, read and written natively.

The TF1 consensus modules publish every model with ``scipy.io.savemat`` and load every
neighbour's with ``scipy.io.loadmat`` (TF1/consensus/cfa.py:108-117, 131-139,
cfa_ongraphs.py:214-223, 282-291, cfa_ge_2stage.py:537-606). ``savemat`` / ``loadmat`` return
the same things as scipy for the files this exchange uses (real numeric arrays and scalars),
through libcfa's level-5 codec (``csrc/cfa_matfile.cpp``):

- ``savemat(path, mdict)`` applies scipy's conversions (Python int -> int64, float -> float64,
  1-D -> a (1, n) row, 0-d -> (1, 1), names starting with '_' skipped) and writes the bytes
  scipy writes (only the header's creation time differs);
- ``loadmat(path)`` returns scipy's dict: '__header__', '__version__', '__globals__' and each
  variable as an array with the file's dims and stored element type (column-major, as scipy
  returns them).

Anything else (compressed files, cells, structs, strings, complex, sparse, bools, empty arrays)
is handed to scipy unchanged, so the result is always scipy's.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import scipy.io as sio

from . import _lib

MI_OF = {np.dtype(np.int8): 1, np.dtype(np.uint8): 2, np.dtype(np.int16): 3, np.dtype(np.uint16): 4,
         np.dtype(np.int32): 5, np.dtype(np.uint32): 6, np.dtype(np.float32): 7, np.dtype(np.float64): 9,
         np.dtype(np.int64): 12, np.dtype(np.uint64): 13}
MX_OF = {np.dtype(np.float64): 6, np.dtype(np.float32): 7, np.dtype(np.int8): 8, np.dtype(np.uint8): 9,
         np.dtype(np.int16): 10, np.dtype(np.uint16): 11, np.dtype(np.int32): 12, np.dtype(np.uint32): 13,
         np.dtype(np.int64): 14, np.dtype(np.uint64): 15}
DTYPE_OF_MI = {v: k for k, v in MI_OF.items()}
MAX_DIM = 8


class MatVar(ctypes.Structure):
    """cfa_mat_var_t"""
    _fields_ = [("name", ctypes.c_char_p), ("mat_class", ctypes.c_int), ("mi_type", ctypes.c_int),
                ("ndim", ctypes.c_int), ("dims", ctypes.c_int64 * MAX_DIM), ("data", ctypes.c_void_p),
                ("nbytes", ctypes.c_size_t)]


def _writeable(value):
    """scipy's to_writeable + oned_as='row' for the values this codec writes, or None."""
    if isinstance(value, bool) or isinstance(value, np.bool_):
        return None
    if isinstance(value, (int, float, np.ndarray, np.generic)):
        a = np.asarray(value)
    else:
        return None
    if a.dtype not in MI_OF or a.size == 0 or a.ndim > MAX_DIM:
        return None
    if a.ndim == 0:
        a = a.reshape(1, 1)
    elif a.ndim == 1:
        a = a.reshape(1, -1)
    return np.asfortranarray(a)


def savemat(path: str, mdict: dict) -> None:
    """scipy.io.savemat(path, mdict) for the TF1 exchange files (see the module docstring)."""
    names, arrays = [], []
    for name, value in mdict.items():
        if not isinstance(name, str) or not name or not name.isidentifier() or len(name) > 63:
            return sio.savemat(path, mdict)
        if name[0] == "_":
            continue  # scipy skips these too
        a = _writeable(value)
        if a is None:
            return sio.savemat(path, mdict)
        names.append(name.encode("latin1"))
        arrays.append(a)
    table = (MatVar * max(1, len(arrays)))()
    for v, name, a in zip(table, names, arrays):
        v.name = name
        v.mat_class = MX_OF[a.dtype]
        v.mi_type = MI_OF[a.dtype]
        v.ndim = a.ndim
        for k, d in enumerate(a.shape):
            v.dims[k] = d
        v.data = a.ctypes.data
        v.nbytes = a.nbytes
    header = "MATLAB 5.0 MAT-file Platform: {}, Created on: {}".format(os.name, time.asctime()).encode("latin1")
    _lib.call("cfa_mat_write", os.fsencode(path), header, len(arrays), table)


def loadmat(path: str) -> dict:
    """scipy.io.loadmat(path) for the TF1 exchange files (see the module docstring)."""
    lib = _lib.load()
    handle = ctypes.c_void_p()
    rc = lib.cfa_mat_read(os.fsencode(path), ctypes.byref(handle))
    if rc == _lib.CFA_E_UNSUPPORTED:
        return sio.loadmat(path)
    if rc != _lib.CFA_OK:
        msg = lib.cfa_last_error()
        raise _lib.CFAError("cfa_mat_read", rc, msg.decode() if msg else "")
    try:
        n = lib.cfa_mat_num_vars(handle)
        vars_ = ctypes.cast(lib.cfa_mat_vars(handle), ctypes.POINTER(MatVar))
        out = {"__header__": lib.cfa_mat_header(handle), "__version__": "1.0", "__globals__": []}
        for i in range(n):
            v = vars_[i]
            dt = DTYPE_OF_MI[v.mi_type]
            shape = tuple(v.dims[k] for k in range(v.ndim))
            raw = ctypes.string_at(v.data, v.nbytes) if v.nbytes else b""
            out[v.name.decode("latin1")] = np.ndarray(shape, dtype=dt, buffer=bytearray(raw), order="F")
        return out
    finally:
        lib.cfa_mat_free(handle)
