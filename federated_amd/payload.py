"""MQTT model payloads: the bytes FL_over_MQTT publishes, decoded and encoded
by libcfa's native codec (``csrc/cfa_payload.cpp``) instead of pickle + Python floats.

The reference publishes ``pickle.dumps({'model_layer{k}': w_k.tolist(), 'device': i,
'framecount': f, 'local_epoch': e, 'training_end': b})`` (TF2/FL_over_MQTT/
learner_consensus.py:257-268; the PS answers with ``global_model_layer{k}``,
``global_epoch``, ``training_end``, PS_server.py:137-149) and reads a payload back with
``st = pickle.loads(payload)`` and ``np.asarray(st['model_layer{k}'])`` per layer
(learner_consensus.py:136-144, PS_server.py:90-118). That builds one Python float object per
parameter, twice per hop.

* ``Payload(data)`` parses the bytes once; ``payload.array(key)`` equals
  ``np.asarray(pickle.loads(data)[key])`` bit for bit (fp64), ``payload.read_into(keys, dst)``
  decodes several layers straight into one flat bucket (e.g. the pinned staging of a mix).
* ``dumps(d)`` returns the exact bytes of ``pickle.dumps({k: v.tolist() ...})`` for ndarray
  values (protocol 4 by default, as CPython 3.10's ``pickle.dumps``), so reference peers read
  them unchanged.
* Only plain containers and scalars are decoded; a payload holding object-constructing pickle
  opcodes is refused (nothing in it is executed).
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from . import _lib

DEFAULT_PROTOCOL = 4  # pickle.DEFAULT_PROTOCOL of the reference's CPython 3.8-3.13


class Payload:
    """A parsed payload. Keeps a reference to the bytes it points into."""

    def __init__(self, data):
        self._buf = np.frombuffer(data, dtype=np.uint8)  # zero-copy view of bytes/bytearray
        self._h = ctypes.c_void_p()
        _lib.call("cfa_payload_parse", self._buf.ctypes.data if self._buf.size else None, self._buf.size,
                  ctypes.byref(self._h))

    def close(self) -> None:
        if self._h:
            _lib.load().cfa_payload_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def keys(self) -> List[str]:
        n = _lib.load().cfa_payload_num_keys(self._h)
        if n < 0:
            _lib.call("cfa_payload_num_keys", self._h)
        out = []
        for i in range(n):
            p, ln = ctypes.c_void_p(), ctypes.c_size_t()
            _lib.call("cfa_payload_key", self._h, i, ctypes.byref(p), ctypes.byref(ln))
            out.append(ctypes.string_at(p, ln.value).decode("utf-8"))
        return out

    def info(self, key: str):
        """(kind, shape) of ``key``'s value; kind is one of _lib.PAYLOAD_*."""
        kind, ndim, numel = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
        shape = (ctypes.c_int64 * _lib.CFA_PAYLOAD_MAX_DIM)()
        _lib.call("cfa_payload_info", self._h, key.encode(), ctypes.byref(kind), ctypes.byref(ndim), shape,
                  ctypes.byref(numel))
        return kind.value, tuple(shape[i] for i in range(ndim.value))

    def scalar(self, key: str):
        """None / bool / int / float value of ``key`` (as pickle.loads returns it)."""
        kind, iv, fv = ctypes.c_int(), ctypes.c_int64(), ctypes.c_double()
        _lib.call("cfa_payload_scalar", self._h, key.encode(), ctypes.byref(kind), ctypes.byref(iv),
                  ctypes.byref(fv))
        k = kind.value
        if k == _lib.PAYLOAD_NONE:
            return None
        if k == _lib.PAYLOAD_BOOL:
            return bool(iv.value)
        if k == _lib.PAYLOAD_INT:
            return int(iv.value)
        return float(fv.value)

    def array(self, key: str, dtype=None, out: Optional[np.ndarray] = None) -> np.ndarray:
        """``np.asarray(value)`` of a (nested) list: fp64 for float lists (int64 / bool for
        lists of ints / bools); ``dtype=np.float32`` returns that array cast to fp32."""
        kind, shape = self.info(key)
        if kind in (_lib.PAYLOAD_STR, _lib.PAYLOAD_DICT, _lib.PAYLOAD_NONE):
            raise TypeError(f"payload key {key!r} is not numeric")
        want = np.dtype(dtype) if dtype is not None else (
            np.dtype(np.float64) if kind in (_lib.PAYLOAD_F64_ARRAY, _lib.PAYLOAD_FLOAT) else None)
        if want is None:  # int / bool lists and scalars: exact through fp64 only below 2**53
            vals = self.array(key, np.float64)
            return vals.astype(np.int64 if kind in (_lib.PAYLOAD_I64_ARRAY, _lib.PAYLOAD_INT) else np.bool_)
        if want not in (np.float64, np.float32):
            raise TypeError("payload arrays decode to float64 or float32")
        if out is None:
            out = np.empty(shape, dtype=want)
        elif out.dtype != want or out.size != int(np.prod(shape)) or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous array of the value's size and dtype")
        fn = "cfa_payload_read_f64" if want == np.float64 else "cfa_payload_read_f32"
        _lib.call(fn, self._h, key.encode(), out.ctypes.data if out.size else None, out.size)
        return out

    def read_into(self, keys: Sequence[str], dst: np.ndarray) -> np.ndarray:
        """Decode the values of ``keys`` back to back (row-major each) into the flat fp64/fp32
        array ``dst`` (e.g. a pinned staging bucket); returns ``dst``."""
        if dst.ndim != 1 or not dst.flags.c_contiguous or dst.dtype not in (np.float64, np.float32):
            raise ValueError("dst must be a contiguous 1-D float64/float32 array")
        fn = "cfa_payload_read_f64" if dst.dtype == np.float64 else "cfa_payload_read_f32"
        pos = 0
        for k in keys:
            _, shape = self.info(k)
            n = int(np.prod(shape))
            if pos + n > dst.size:
                raise ValueError("dst is smaller than the decoded layers")
            _lib.call(fn, self._h, k.encode(), dst.ctypes.data + pos * dst.itemsize if n else None, n)
            pos += n
        if pos != dst.size:
            raise ValueError(f"decoded {pos} values into a bucket of {dst.size}")
        return dst

    def to_dict(self) -> Dict[str, object]:
        """{key: np.asarray(list) | scalar}: what the reference holds after pickle.loads and
        np.asarray on the layer lists."""
        out = {}
        for k in self.keys():
            kind, _ = self.info(k)
            if kind in (_lib.PAYLOAD_F64_ARRAY, _lib.PAYLOAD_I64_ARRAY, _lib.PAYLOAD_BOOL_ARRAY):
                out[k] = self.array(k)
            elif kind in (_lib.PAYLOAD_STR, _lib.PAYLOAD_DICT):
                raise TypeError(f"payload key {k!r}: strings / nested dicts are not decoded")
            else:
                out[k] = self.scalar(k)
        return out


def loads(data) -> Dict[str, object]:
    """``{k: np.asarray(v) if list else v for k, v in pickle.loads(data).items()}``."""
    with Payload(data) as p:
        return p.to_dict()


def _item(key: str, value, keep):
    it = _lib.PayloadItem()
    it.key = key.encode("utf-8")
    keep.append(it.key)
    if isinstance(value, np.ndarray):
        a = value
        if a.dtype not in (np.float32, np.float64):
            raise TypeError(f"{key!r}: only float32/float64 arrays are encoded (tolist floats)")
        a = a if a.flags.c_contiguous else a.copy(order="C")  # (ascontiguousarray makes 0-d 1-d)
        if a.ndim > _lib.CFA_PAYLOAD_MAX_DIM:
            raise ValueError(f"{key!r}: more than {_lib.CFA_PAYLOAD_MAX_DIM} dimensions")
        shape = _lib.int64_array(a.shape)
        keep.extend([a, shape])
        it.kind = _lib.PAYLOAD_F32_ARRAY if a.dtype == np.float32 else _lib.PAYLOAD_F64_ARRAY
        it.data = a.ctypes.data
        it.ndim = a.ndim
        it.shape = ctypes.cast(shape, ctypes.POINTER(ctypes.c_int64))
    elif value is None:
        it.kind = _lib.PAYLOAD_NONE
    elif isinstance(value, (bool, np.bool_)):
        it.kind, it.ivalue = _lib.PAYLOAD_BOOL, int(bool(value))
    elif isinstance(value, int):
        if not -(1 << 63) <= value < (1 << 63):
            raise OverflowError(f"{key!r}: integer wider than 64 bits")
        it.kind, it.ivalue = _lib.PAYLOAD_INT, value
    elif isinstance(value, float):
        it.kind, it.fvalue = _lib.PAYLOAD_FLOAT, value
    else:
        raise TypeError(f"{key!r}: {type(value).__name__} values are not encoded "
                        "(ndarray, int, bool, float, None)")
    return it


def _items(d: Dict[str, object], keep: List[object]):
    items = (_lib.PayloadItem * max(1, len(d)))()
    for i, (k, v) in enumerate(d.items()):
        items[i] = _item(k, v, keep)
    return items


_bytes_new = ctypes.pythonapi.PyBytes_FromStringAndSize
_bytes_new.restype = ctypes.py_object
_bytes_new.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]


def dumps(d: Dict[str, object], protocol: int = DEFAULT_PROTOCOL) -> bytes:
    """Bytes of ``pickle.dumps({k: (v.tolist() if ndarray else v)}, protocol)``. The encoder
    writes straight into a fresh (not yet shared) bytes object: no intermediate copy."""
    keep: List[object] = []
    items = _items(d, keep)
    size = ctypes.c_size_t()
    _lib.call("cfa_payload_encode", items, len(d), protocol, None, 0, ctypes.byref(size))
    out = _bytes_new(None, size.value)
    addr = ctypes.cast(ctypes.c_char_p(out), ctypes.c_void_p).value
    _lib.call("cfa_payload_encode", items, len(d), protocol, addr, size.value, ctypes.byref(size))
    return out


def dumps_into(d: Dict[str, object], buf, protocol: int = DEFAULT_PROTOCOL) -> int:
    """Encode into a caller-owned writable buffer (bytearray / uint8 ndarray, reused across
    publishes); returns the byte count. Raises if the buffer is too small."""
    keep: List[object] = []
    items = _items(d, keep)
    view = np.frombuffer(buf, dtype=np.uint8)
    if not view.flags.writeable:
        raise ValueError("buffer is read-only")
    size = ctypes.c_size_t()
    _lib.call("cfa_payload_encode", items, len(d), protocol, None, 0, ctypes.byref(size))
    if size.value > view.size:
        raise ValueError(f"buffer holds {view.size} bytes, the payload needs {size.value}")
    _lib.call("cfa_payload_encode", items, len(d), protocol, view.ctypes.data, view.size, ctypes.byref(size))
    return size.value


def encoded_size(d: Dict[str, object], protocol: int = DEFAULT_PROTOCOL) -> int:
    keep: List[object] = []
    size = ctypes.c_size_t()
    _lib.call("cfa_payload_encode", _items(d, keep), len(d), protocol, None, 0, ctypes.byref(size))
    return size.value


def layer_keys(prefix: str, layers: int) -> List[str]:
    """['model_layer0', ...] (learner_consensus.py:143, 262) / 'global_model_layer{k}'
    (PS_server.py:142)."""
    return [f"{prefix}{k}" for k in range(layers)]


def model_payload(weights: Iterable[np.ndarray], prefix: str = "model_layer", **scalars) -> bytes:
    """The learner's publish (learner_consensus.py:261-268): layer lists then the scalars in
    the caller's order, e.g. ``model_payload(w, device=i, framecount=f, local_epoch=e,
    training_end=b)``."""
    d: Dict[str, object] = {}
    for k, w in enumerate(weights):
        d[f"{prefix}{k}"] = np.asarray(w)
    d.update(scalars)
    return dumps(d)
