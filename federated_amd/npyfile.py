"""numpy files of the TF2 exchange, read natively.

The TF2 consensus and parameter-server modules load every neighbour's status archive and model
with ``np.load(path, allow_pickle=True)`` (TF2/MNIST_dataset/consensus/consensus_v3.py:82-141,
consensus_v4.py:30-95, parameter_server_v2.py:83-164):

- ``results/dump_train_variables{k}.npz``: ``np.savez`` of 0-d numeric arrays (stored zip);
- ``results/dump_train_model{k}.npy``: ``np.save`` of the Keras weight list as a 1-D object
  array, which numpy writes as a pickle.

``load(path)`` returns what ``np.load(path, allow_pickle=True)`` returns for these files, through
libcfa's reader (``csrc/cfa_npy.cpp``): the file is read once into a numpy-owned buffer, libcfa
locates the arrays in it (walking an object array's pickle without executing anything from it),
and the arrays come back as writeable views of that buffer. An ``.npz`` comes back as a
read-only mapping of member name -> array (``NpzFile``'s ``[]``, ``files``, ``keys()``, ``in``,
``close()`` and ``with``). Files outside the reader's scope (compressed archives, structured or
big-endian dtypes, other pickled objects) go to ``np.load`` unchanged; a truncated or corrupt
file raises, as ``np.load`` does.

``load(path, slot=key)`` reads into a per-thread buffer kept under ``key`` instead of a fresh one
(no page faults on every read): the arrays it returns are valid only until the next load with
the same key on the same thread. The drop-in's neighbour loops use it for the models they
consume within the call (the mix copies them out); anything handed back to the caller is copied.
"""
from __future__ import annotations

import ctypes
import os
import threading
from collections.abc import Mapping

import numpy as np

from . import _lib

MAX_DIM = 32
ARRAY, OBJECT, ARCHIVE = 0, 1, 2


class NpyArray(ctypes.Structure):
    """cfa_npy_array_t"""
    _fields_ = [("name", ctypes.c_char_p), ("descr", ctypes.c_char_p), ("itemsize", ctypes.c_int),
                ("ndim", ctypes.c_int), ("shape", ctypes.c_int64 * MAX_DIM), ("fortran_order", ctypes.c_int),
                ("data", ctypes.c_void_p), ("nbytes", ctypes.c_size_t)]


class Archive(Mapping):
    """The members of an ``.npz`` (what ``np.load`` returns for one, as a mapping)."""

    def __init__(self, members: dict):
        self._members = members
        self.files = list(members)

    def __getitem__(self, key):
        return self._members[key]

    def __iter__(self):
        return iter(self._members)

    def __len__(self):
        return len(self._members)

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


_tls = threading.local()


def _slot_buffer(slot, size: int) -> np.ndarray:
    bufs = getattr(_tls, "bufs", None)
    if bufs is None:
        bufs = _tls.bufs = {}
    b = bufs.get(slot)
    if b is None or b.size < size:
        if len(bufs) >= 64:  # bounded: one buffer per neighbour slot in practice
            bufs.clear()
        b = bufs[slot] = np.empty(size + (size >> 3), dtype=np.uint8)  # headroom for growing files
    return b[:size]


def _read_image(path, slot=None) -> np.ndarray:
    """The file's bytes in one unbuffered read into an uninitialised numpy buffer (numpy's
    allocator: no zero-fill pass over fresh pages, unlike bytearray(n)), or into the slot's
    reused buffer."""
    with open(path, "rb", buffering=0) as f:
        size = os.fstat(f.fileno()).st_size
        image = np.empty(size, dtype=np.uint8) if slot is None else _slot_buffer(slot, size)
        got = f.readinto(image) if size else 0
    return image[:got] if got != size else image


def load(path, slot=None):
    """np.load(path, allow_pickle=True) for the TF2 exchange files (see the module docstring)."""
    image = _read_image(path, slot)
    lib = _lib.load()
    handle = ctypes.c_void_p()
    start = image.ctypes.data
    rc = lib.cfa_npy_parse(start if image.size else None, image.size, ctypes.byref(handle))
    if rc == _lib.CFA_E_UNSUPPORTED:
        return np.load(path, allow_pickle=True)
    if rc != _lib.CFA_OK:
        msg = lib.cfa_last_error()
        raise _lib.CFAError("cfa_npy_parse", rc, msg.decode() if msg else "")
    try:
        kind = lib.cfa_npy_kind(handle)
        n = lib.cfa_npy_num_arrays(handle)
        recs = ctypes.cast(lib.cfa_npy_arrays(handle), ctypes.POINTER(NpyArray))
        arrays, names = [], []
        for i in range(n):
            r = recs[i]
            shape = tuple(r.shape[k] for k in range(r.ndim))
            a = np.ndarray(shape, dtype=np.dtype(r.descr.decode()), buffer=image,
                           offset=(r.data - start) if r.nbytes else 0, order="F" if r.fortran_order else "C")
            arrays.append(a)
            names.append(r.name.decode() if r.name else None)
    finally:
        lib.cfa_npy_free(handle)
    if kind == ARRAY:
        return arrays[0]
    if kind == OBJECT:
        out = np.empty(len(arrays), dtype=object)
        for i, a in enumerate(arrays):
            out[i] = a
        return out
    return Archive(dict(zip(names, arrays)))
