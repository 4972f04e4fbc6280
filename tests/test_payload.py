"""(f2) MQTT payload codec (libcfa cfa_payload_*), host-only: no GPU needed.

The reference's codec is CPython's stdlib pickle applied to the dicts its FL_over_MQTT drivers
build (learner_consensus.py:257-268, PS_server.py:137-149) and np.asarray on the decoded layer
lists (learner_consensus.py:136-144, PS_server.py:90-118); ``oracle.cfa_oracle.mqtt_*``
restate those lines. Encoding must give the same BYTES, decoding the same fp64 VALUES (bit
patterns, NaN payloads included).
"""
import pickle

import numpy as np
import pytest

from federated_amd import _lib
from federated_amd import payload as pl
from federated_amd import server
from oracle import cfa_oracle as orc

# TF2 radar CNN (FL_radar_dataset ...consensus_FL.py:158-172) and the MQTT learner's CNN
# (learner_consensus.py:108-124: Conv2D(4,5x5) on (256,63,1), Conv2D(8,5x5), Dense(n_outputs))
RADAR = [(8, 8, 1, 32), (32,), (4, 4, 32, 64), (64,), (3, 3, 64, 64), (64,), (7168, 512), (512,), (512, 6), (6,)]
MQTT_CNN = [(5, 5, 1, 4), (4,), (5, 5, 4, 8), (8,), (7200, 6), (6,)]


def _model(shapes, seed, dtype=np.float32):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(s).astype(dtype) for s in shapes]


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def _tolist_dict(d):
    return {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in d.items()}


# ---------------------------------------------------------------------------------------------
# encoder: byte identity with pickle.dumps
# ---------------------------------------------------------------------------------------------

def test_learner_and_ps_payload_bytes_match_the_reference():
    w = _model(MQTT_CNN, 1)
    assert server.learner_publish(w, 3, 1234, 17, False) == orc.mqtt_learner_payload(w, 3, 1234, 17, False)
    assert server.learner_publish(w, 0, 0, 0, True) == orc.mqtt_learner_payload(w, 0, 0, 0, True)
    assert server.ps_mqtt_publish(w, 42, False) == orc.mqtt_ps_payload(w, 42, False)


def test_radar_payload_bytes_match_the_reference():
    w = _model(RADAR, 2)  # 3.7M params: 33.7 MB, 515 frames, threaded float blocks
    assert server.learner_publish(w, 7, 99, 5, False) == orc.mqtt_learner_payload(w, 7, 99, 5, False)


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_random_structures_bytes_match_pickle(protocol):
    rng = np.random.default_rng(100 + protocol)
    for _ in range(60):
        d = {}
        for k in range(int(rng.integers(1, 6))):
            nd = int(rng.integers(0, 5))
            if rng.random() < 0.7:
                shape = tuple(int(x) for x in rng.integers(0 if rng.random() < 0.15 else 1, 12, size=nd))
            else:
                shape = (int(rng.integers(1, 30000)),)
            a = rng.standard_normal(shape).astype(np.float32 if rng.random() < 0.6 else np.float64)
            if a.ndim > 1 and rng.random() < 0.3:
                a = a.T  # non-contiguous source
            d[f"model_layer{k}"] = a
        d["device"] = int(rng.integers(-(10 ** 15), 10 ** 15)) if rng.random() < 0.3 else int(rng.integers(0, 70000))
        d["training_end"] = bool(rng.integers(0, 2))
        d["lr"] = float(rng.standard_normal())
        d["none"] = None
        assert pl.dumps(d, protocol) == pickle.dumps(_tolist_dict(d), protocol)


@pytest.mark.parametrize("value", [0, 1, 255, 256, 65535, 65536, -1, -128, -129, 2 ** 31 - 1, 2 ** 31, -2 ** 31,
                                   -2 ** 31 - 1, 2 ** 40, -2 ** 40, 2 ** 63 - 1, -2 ** 63, 127, 128, 32767, 32768])
def test_integer_encodings(value):
    for protocol in (2, 4):
        assert pl.dumps({"i": value}, protocol) == pickle.dumps({"i": value}, protocol)


def test_edge_structures():
    cases = [
        {},
        {"a": np.zeros((0,), np.float32)},
        {"a": np.zeros((3, 0), np.float32), "b": np.zeros((0, 3), np.float64)},
        {"a": np.ones((), np.float32)},  # 0-d: tolist() is a float
        {"a": np.ones((1,), np.float32), "b": np.ones((1, 1, 1), np.float32)},  # APPEND path
        {"a": np.ones((1000,), np.float32), "b": np.ones((1001,), np.float32), "c": np.ones((999,))},
        {"a": np.array([np.nan, np.inf, -np.inf, -0.0, 0.0, 1e-45, 3.4e38], np.float32)},
        {"a": np.array([np.nan, 5e-324, -1.7976931348623157e308], np.float64)},
        {"k" * 300: 1.5, "ü-key": True},  # BINUNICODE (>255 bytes), non-ASCII
        {f"key{i}": i for i in range(2500)},  # SETITEMS batches of 1000
        {"a": np.zeros((400, 2), np.float32)},  # > 256 memo entries (LONG_BINPUT in protocol 2)
        {"a": np.zeros((7281,)), "b": np.zeros((1,))},  # frame commit right before a small item
    ]
    for d in cases:
        for protocol in (2, 3, 4, 5):
            assert pl.dumps(d, protocol) == pickle.dumps(_tolist_dict(d), protocol), (list(d)[:3], protocol)


def test_frame_boundaries_sweep():
    """Frames commit before the object that finds >= 64 KiB in the current frame: sweep the
    header length so the boundary lands at every offset of a 9-byte BINFLOAT record."""
    for pad in range(0, 40):
        d = {"p" * (pad + 1): 1, "a": np.arange(20000, dtype=np.float32).reshape(100, 200)}
        assert pl.dumps(d) == pickle.dumps(_tolist_dict(d))


def test_dumps_into_and_size():
    d = {"model_layer0": np.ones((10, 10), np.float32), "device": 1}
    ref = pickle.dumps(_tolist_dict(d))
    assert pl.encoded_size(d) == len(ref)
    buf = bytearray(len(ref) + 10)
    n = pl.dumps_into(d, buf)
    assert n == len(ref) and bytes(buf[:n]) == ref
    with pytest.raises(ValueError):
        pl.dumps_into(d, bytearray(len(ref) - 1))


def test_encoder_refuses_what_it_cannot_reproduce():
    for bad in ({"a": np.ones(3, np.int64)}, {"a": np.float32(1.0)}, {"a": "text"}, {"a": [1.0, 2.0]},
                {"a": 2 ** 64}):
        with pytest.raises((TypeError, OverflowError)):
            pl.dumps(bad)


# ---------------------------------------------------------------------------------------------
# decoder: values of np.asarray(pickle.loads(...)[key])
# ---------------------------------------------------------------------------------------------

def test_decode_learner_payload_equals_reference_decode():
    w = _model(MQTT_CNN, 3)
    data = orc.mqtt_learner_payload(w, 5, 10, 2, False)
    ref = orc.mqtt_decode_layers(data, len(w))
    with pl.Payload(data) as p:
        got = [p.array(f"model_layer{k}") for k in range(len(w))]
        assert p.keys() == list(pickle.loads(data).keys())
        assert (p.scalar("device"), p.scalar("framecount"), p.scalar("local_epoch"), p.scalar("training_end")) \
            == (5, 10, 2, False)
        for k in range(len(w)):
            f32 = p.array(f"model_layer{k}", np.float32)
            assert _bits_equal(f32, ref[k].astype(np.float32))
    for a, r in zip(got, ref):
        assert _bits_equal(a, r)


def test_decode_radar_payload_threaded_and_into_bucket():
    w = _model(RADAR, 4)
    data = orc.mqtt_learner_payload(w, 1, 2, 3, True)
    ref = orc.mqtt_decode_layers(data, len(w))
    flat_ref = np.concatenate([r.reshape(-1) for r in ref])
    p = pl.Payload(data)
    dst = np.empty(flat_ref.size, np.float64)
    p.read_into(pl.layer_keys("model_layer", len(w)), dst)
    assert dst.tobytes() == flat_ref.tobytes()
    dst32 = np.empty(flat_ref.size, np.float32)
    p.read_into(pl.layer_keys("model_layer", len(w)), dst32)
    assert dst32.tobytes() == flat_ref.astype(np.float32).tobytes()
    with pytest.raises(ValueError):
        p.read_into(pl.layer_keys("model_layer", len(w)), np.empty(flat_ref.size + 1))


@pytest.mark.parametrize("protocol", [2, 3, 4, 5])
def test_decode_stdlib_pickles(protocol):
    shared = [1.5, 2.5]
    obj = {
        "floats": [[0.5, -0.0, float("nan")], [float("inf"), 1e-310, -3.0]],
        "ints": [1, -2, 3 * 10 ** 12, 255, 65536],
        "bools": [True, False],
        "mixed": [1, 2.5, True],
        "shared": [shared, shared],  # memo GET of a list
        "empty": [],
        "nested_empty": [[], []],
        "one": [[7.0]],
        "scalar_f": 0.25, "scalar_i": -7, "scalar_b": True, "none": None,
        "big": np.linspace(-1, 1, 5000).tolist(),
    }
    data = pickle.dumps(obj, protocol)
    got = pl.loads(data)
    assert list(got) == list(obj)
    for k, v in obj.items():
        if isinstance(v, list):
            assert _bits_equal(got[k], np.asarray(v)), k
        else:
            assert got[k] == v and type(got[k]) is type(v), k


def test_ragged_and_non_numeric_lists_are_errors():
    for obj in ({"a": [[1.0], [1.0, 2.0]]}, {"a": [[1.0], 2.0]}, {"a": ["x"]}, {"a": [None]}):
        with pl.Payload(pickle.dumps(obj)) as p:
            with pytest.raises(_lib.CFAError):
                p.array("a")


def test_object_constructing_payloads_are_refused():
    """Nothing in a payload is executed: object-constructing opcodes fail the parse."""
    payloads = [
        pickle.dumps({"a": np.float32(1.0)}),            # numpy scalar: STACK_GLOBAL + REDUCE
        pickle.dumps({"a": np.ones(3)}),                 # ndarray reconstruct
        b"\x80\x04}\x94\x8c\x01a\x94cos\nsystem\n\x94s.",  # GLOBAL os.system
        pickle.dumps({"a": (1.0, 2.0)}),                 # tuples are not model payload values
        b"(lp0\nF1.0\na.",                               # protocol 0 text opcodes
    ]
    for data in payloads:
        with pytest.raises(_lib.CFAError):
            pl.Payload(data)


def test_truncated_payloads_fail_cleanly():
    data = orc.mqtt_learner_payload(_model([(3, 4), (4,)], 5), 1, 2, 3, False)
    for cut in range(len(data)):
        with pytest.raises(_lib.CFAError):
            pl.Payload(data[:cut])
    pl.Payload(data)


def test_corrupted_payloads_never_crash():
    rng = np.random.default_rng(7)
    data = orc.mqtt_learner_payload(_model([(3, 4), (4,), (2, 2)], 6), 1, 2, 3, False)
    for _ in range(3000):
        b = bytearray(data)
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        try:
            p = pl.Payload(bytes(b))
        except _lib.CFAError:
            continue
        try:  # pickle.loads raises UnicodeDecodeError for a corrupted key as well
            p.to_dict()
        except (_lib.CFAError, TypeError, UnicodeDecodeError):
            pass


def test_round_trip():
    w = _model(MQTT_CNN, 8, np.float64)
    d = {f"model_layer{k}": a for k, a in enumerate(w)}
    d.update(device=1, training_end=False)
    back = pl.loads(pl.dumps(d))
    for k, a in enumerate(w):
        assert _bits_equal(back[f"model_layer{k}"], a)
    assert back["device"] == 1 and back["training_end"] is False


def test_codec_under_address_sanitizer():
    """The codec's host code built with -fsanitize=address,undefined and fuzzed with mutated and
    truncated reference payloads (tools/asan/run_payload_fuzz.sh)."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "asan",
                          "run_payload_fuzz.sh")
    r = subprocess.run(["bash", script, "3000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "no finding" in r.stdout
