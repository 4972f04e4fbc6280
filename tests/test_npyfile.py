"""libcfa's numpy reader (federated_amd/npyfile.py, csrc/cfa_npy.cpp) against np.load, which the
reference's TF2 exchange calls on every neighbour's status archive and model
(TF2/MNIST_dataset/consensus/consensus_v3.py:82-141, consensus_v4.py:30-95,
parameter_server_v2.py:83-164; the drivers write them with np.savez / np.save of
np.asarray(model.get_weights()), e.g. FL_radar_dataset/federated_learning_keras_PS.py:264-268).
Every in-scope file must load to np.load's arrays (dtype, shape, order, values); everything
else must reach np.load unchanged. CPU only (no GPU call)."""
import ctypes
import io
import os
import pickle

import numpy as np
import pytest

from federated_amd import _lib, npyfile

rng = np.random.default_rng(5)

VGG1 = [(3, 3, 3, 32), (32,), (3, 3, 32, 32), (32,), (8192, 128), (128,), (128, 100), (100,)]


def objarr(arrays):
    out = np.empty(len(arrays), dtype=object)
    for i, a in enumerate(arrays):
        out[i] = a
    return out


def write_object_npy(f, arr, protocol):
    """np.save's layout (format 1.0 header, then a pickle of the array) at a chosen pickle protocol."""
    np.lib.format.write_array_header_1_0(f, np.lib.format.header_data_from_array_1_0(arr))
    pickle.dump(arr, f, protocol=protocol)


def keras_weights(shapes, dtype=np.float32):
    return objarr([rng.standard_normal(s).astype(dtype) for s in shapes])


def same(a, b):
    assert type(a) is type(b) or isinstance(b, npyfile.Archive)
    if isinstance(b, npyfile.Archive):
        assert list(a.files) == list(b.files)
        for k in a.files:
            same(a[k], b[k])
        return
    assert a.dtype == b.dtype and a.shape == b.shape, (a.dtype, b.dtype, a.shape, b.shape)
    if a.dtype == object:
        for x, y in zip(a.ravel(), b.ravel()):
            same(x, y)
        return
    assert a.flags.f_contiguous == b.flags.f_contiguous
    assert a.flags.c_contiguous == b.flags.c_contiguous
    np.testing.assert_array_equal(a, b)


def native_kind(path):
    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.cfa_npy_read(os.fsencode(str(path)), ctypes.byref(h))
    if rc == 0:
        k = lib.cfa_npy_kind(h)
        lib.cfa_npy_free(h)
        return k
    return rc


OBJECT_CASES = {
    "vgg1_f32": lambda: keras_weights(VGG1),
    "radar_cnn": lambda: keras_weights([(8, 8, 1, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,),
                                        (7168, 64), (64,), (64, 6), (6,)]),
    "lenet_f64": lambda: keras_weights([(5, 5, 1, 6), (6,), (400, 10), (10,)], np.float64),
    "mixed": lambda: objarr([np.arange(6, dtype=np.int32).reshape(2, 3), np.ones((3, 2), np.float32).T,
                             np.array(2.5), np.zeros((0, 4), np.float32), np.array([True, False]),
                             np.arange(5, dtype=np.uint8), np.arange(3, dtype=np.float16),
                             np.arange(4, dtype=np.int64), np.arange(4, dtype=np.uint64)]),
    "one_layer": lambda: objarr([np.ones(3, np.float32)]),
    "empty": lambda: np.empty(0, dtype=object),
}


@pytest.mark.parametrize("case", sorted(OBJECT_CASES))
def test_object_arrays_match_np_load(case, tmp_path):
    p = tmp_path / "dump_train_model0.npy"
    np.save(p, OBJECT_CASES[case](), allow_pickle=True)
    assert native_kind(p) == npyfile.OBJECT
    same(np.load(p, allow_pickle=True), npyfile.load(str(p)))


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_pickle_protocols(protocol, tmp_path):
    p = tmp_path / "m.npy"
    w = OBJECT_CASES["mixed"]()
    with open(p, "wb") as f:
        write_object_npy(f, w, protocol)
    # np.save writes protocol 3 (numpy 1.x) or 4 (numpy 2.x): read natively; 2 and 5 spell the
    # data through other callables (_codecs.encode, _frombuffer) and go to np.load
    assert native_kind(p) == (npyfile.OBJECT if protocol in (3, 4) else _lib.CFA_E_UNSUPPORTED)
    want = np.load(p, allow_pickle=True)
    got = npyfile.load(str(p))
    same(want, got)


def test_numpy1_module_path(tmp_path):
    """numpy 1.x pickles name numpy.core.multiarray (protocol 3, GLOBAL opcode)."""
    buf = io.BytesIO()
    write_object_npy(buf, keras_weights([(4, 3), (3,)]), 3)
    raw = buf.getvalue()
    assert b"numpy._core.multiarray\n_reconstruct" in raw
    p = tmp_path / "old.npy"
    p.write_bytes(raw.replace(b"numpy._core.multiarray\n", b"numpy.core.multiarray\n"))
    assert native_kind(p) == npyfile.OBJECT
    same(np.load(p, allow_pickle=True), npyfile.load(str(p)))


NUMERIC = {
    "f32": np.arange(12, dtype=np.float32).reshape(3, 4),
    "f64_fortran": np.asfortranarray(rng.standard_normal((5, 3))),
    "i64_scalar": np.array(7, dtype=np.int64),
    "bool": np.array([True, False, True]),
    "u8_3d": np.arange(24, dtype=np.uint8).reshape(2, 3, 4),
    "f16": np.arange(5, dtype=np.float16),
    "empty": np.zeros((0, 3), np.float32),
    "same_shape_layers": np.asarray([np.ones((2, 2), np.float32)] * 3),  # np.asarray of equal-shape weights
}


@pytest.mark.parametrize("case", sorted(NUMERIC))
def test_numeric_npy_match_np_load(case, tmp_path):
    p = tmp_path / "a.npy"
    np.save(p, NUMERIC[case])
    assert native_kind(p) == npyfile.ARRAY
    same(np.load(p, allow_pickle=True), npyfile.load(str(p)))


def test_npy_format_v2_header(tmp_path):
    p = tmp_path / "v2.npy"
    with open(p, "wb") as f:
        np.lib.format.write_array(f, np.arange(6.0).reshape(2, 3), version=(2, 0))
    same(np.load(p), npyfile.load(str(p)))


def test_status_archives_match_np_load(tmp_path):
    """The drivers' status file (federated_learning_keras_PS.py:266-267) and the v3 one."""
    p = tmp_path / "dump_train_variables3.npz"
    np.savez(p, frame_count=70000, epoch_loss_history=[0.5, 0.25, 0.125], training_end=False,
             epoch_count=12, loss=0.0625)
    assert native_kind(p) == npyfile.ARCHIVE
    want, got = np.load(p, allow_pickle=True), npyfile.load(str(p))
    same(want, got)
    assert got["epoch_count"] == 12 and bool(got["training_end"]) is False
    with npyfile.load(str(p)) as d:
        assert "loss" in d and d["loss"] == 0.0625 and sorted(d.keys()) == sorted(want.files)
    p2 = tmp_path / "v.npz"
    np.savez(p2, epoch_count=3, training_end=True, empty=np.zeros(0))
    same(np.load(p2, allow_pickle=True), npyfile.load(str(p2)))


@pytest.mark.parametrize("make", ["compressed", "structured", "big_endian", "object_of_lists", "object_2d",
                                  "object_in_npz", "complex", "unicode", "nested_object"])
def test_outside_scope_goes_to_np_load(make, tmp_path):
    p = tmp_path / ("x.npz" if make in ("compressed", "object_in_npz") else "x.npy")
    if make == "compressed":
        np.savez_compressed(p, epoch_count=3, training_end=False)
    elif make == "structured":
        np.save(p, np.zeros(3, dtype=[("a", "<f4"), ("b", "<i4")]))
    elif make == "big_endian":
        np.save(p, np.arange(4, dtype=">f4"))
    elif make == "object_of_lists":
        np.save(p, objarr([[1.0, 2.0], "text"]), allow_pickle=True)
    elif make == "object_2d":
        o = np.empty((2, 1), dtype=object)
        o[0, 0], o[1, 0] = np.ones(2), np.ones(3)
        np.save(p, o, allow_pickle=True)
    elif make == "object_in_npz":
        np.savez(p, w=keras_weights([(2, 2), (2,)]))
    elif make == "complex":
        np.save(p, np.ones(3, np.complex64))
    elif make == "unicode":
        np.save(p, np.array(["ab", "c"]))
    elif make == "nested_object":
        np.save(p, objarr([objarr([np.ones(2)]), np.ones(3)]), allow_pickle=True)
    assert native_kind(p) == _lib.CFA_E_UNSUPPORTED
    want = np.load(p, allow_pickle=True)
    got = npyfile.load(str(p))
    if hasattr(want, "files"):
        assert list(want.files) == list(got.files)
    else:
        assert want.dtype == got.dtype and want.shape == got.shape


def test_pickle_with_foreign_global_executes_nothing(tmp_path):
    """An object .npy whose pickle names any callable other than numpy's reconstructors is refused
    before anything runs (the reader is a parser, not an unpickler)."""
    class Boom:
        def __reduce__(self):
            return (os.getcwd, ())
    p = tmp_path / "evil.npy"
    with open(p, "wb") as f:
        f.write(b"\x93NUMPY\x01\x00")
        header = "{'descr': '|O', 'fortran_order': False, 'shape': (1,), }"
        header += " " * (117 - len(header)) + "\n"
        f.write(len(header).to_bytes(2, "little") + header.encode())
        pickle.dump(objarr([Boom()]), f, protocol=4)
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.cfa_npy_read(os.fsencode(str(p)), ctypes.byref(h)) == _lib.CFA_E_UNSUPPORTED
    assert b"posix.getcwd" in lib.cfa_last_error() or b"getcwd" in lib.cfa_last_error()


def test_truncated_and_corrupt_files_raise(tmp_path):
    """A neighbour's file read while it is being rewritten must raise (the caller retries after
    pause(5), consensus_v3.py:130-141), never return partial arrays."""
    src = tmp_path / "m.npy"
    np.save(src, keras_weights([(64, 8), (8,), (8, 3), (3,)]), allow_pickle=True)
    data = src.read_bytes()
    cut = tmp_path / "cut.npy"
    for n in (0, 5, 9, 60, 128, 200, len(data) // 2, len(data) - 1):
        cut.write_bytes(data[:n])
        with pytest.raises(Exception):
            np.load(cut, allow_pickle=True)
        with pytest.raises(_lib.CFAError):
            npyfile.load(str(cut))
    z = tmp_path / "v.npz"
    np.savez(z, epoch_count=4, training_end=False)
    zb = bytearray(z.read_bytes())
    for n in (0, 10, 30, len(zb) // 2, len(zb) - 1):
        cut.write_bytes(bytes(zb[:n]))
        with pytest.raises(Exception):
            npyfile.load(str(cut))
    i = zb.index(b"\x93NUMPY")  # flip one data byte of the first member: CRC mismatch, as zipfile
    zb[i + 130] ^= 0xFF
    cut.write_bytes(bytes(zb))
    with pytest.raises(_lib.CFAError, match="CRC"):
        npyfile.load(str(cut))
    with pytest.raises(Exception):
        npyfile.load(str(tmp_path / "missing.npy"))


def test_loaded_arrays_are_writeable_and_independent(tmp_path):
    p = tmp_path / "m.npy"
    np.save(p, keras_weights([(4, 3), (3,)]), allow_pickle=True)
    a, b = npyfile.load(str(p)), npyfile.load(str(p))
    a[0][0, 0] = 123.0  # the drop-in writes into loaded layers (training_end copy, consensus_v3.py:147-152)
    assert b[0][0, 0] != 123.0 and npyfile.load(str(p))[0][0, 0] != 123.0


def test_tf2_protocol_uses_reader(tmp_path, monkeypatch):
    """The TF2 drop-in's status and model loads go through the reader, not np.load."""
    from federated_amd.consensus import _tf2
    os.makedirs(tmp_path / "results")
    monkeypatch.chdir(tmp_path)
    np.savez("results/dump_train_variables1.npz", epoch_count=2, training_end=False)
    w = keras_weights([(4, 3), (3,)])
    np.save("results/dump_train_model1.npy", w, allow_pickle=True)
    calls = []
    real = np.load
    monkeypatch.setattr(np, "load", lambda *a, **k: calls.append(a) or real(*a, **k))
    base = _tf2.TF2Base(3, 0, 1)
    ok, count = base._read_status("results/dump_train_variables1.npz")
    model, success = base._wait_and_load("results/dump_train_variables1.npz", "results/dump_train_model1.npy",
                                         count, 2, 30)
    assert ok and count == 2 and success and calls == []
    same(w, model)


def test_reader_under_address_sanitizer():
    """The reader's host code built with -fsanitize=address,undefined and fuzzed with mutated and
    truncated np.save / np.savez files (tools/asan/run_npy_fuzz.sh)."""
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "asan",
                          "run_npy_fuzz.sh")
    r = subprocess.run(["bash", script, "3000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "no finding" in r.stdout


def test_slot_loads_reuse_one_buffer(tmp_path):
    """load(path, slot=k) reads into the slot's reused buffer: same values as a fresh load; the
    arrays of the previous load with that slot are overwritten by the next one (the contract the
    drop-in's neighbour loops rely on), other slots are untouched."""
    a, b = tmp_path / "a.npy", tmp_path / "b.npy"
    wa, wb = keras_weights([(40, 3), (3,)]), keras_weights([(40, 3), (3,)])
    np.save(a, wa, allow_pickle=True)
    np.save(b, wb, allow_pickle=True)
    x = npyfile.load(str(a), slot=("t", 0))
    same(wa, x)
    y = npyfile.load(str(b), slot=("t", 1))
    same(wa, x)  # another slot: x intact
    z = npyfile.load(str(b), slot=("t", 0))
    same(wb, z)
    assert np.shares_memory(x[0], z[0]) and np.array_equal(x[0], wb[0])  # x now shows b's bytes
    same(wb, y)
