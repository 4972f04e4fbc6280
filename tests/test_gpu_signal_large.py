"""The completion word (consensus/_runtime._ZeroCopyPlan.complete) at multi-MB buckets, one test
per zero-copy kind: the kernels' output is written into pinned host memory from every XCD (a
3.1M-element bucket is many chunks of tiles per XCD), and the host reads it right after the
one-lane signal kernel of the same stream has released the word. Each call's result must equal
the staged path (device buffers, explicit D2H copy, hipStreamSynchronize) of the same inputs, bit
for bit, and the calls run back to back on changing inputs, so a wait that returned before the
output was visible would hand back the previous call's values.

Kinds: f32 (TF2 rule with the cfa_ongraphs compression epilogue, and the TF1 rule on fp32
rows), tf1w (TF1 rule on fp32 arrays into an fp64 row), f64 (TF1 rule on fp64 rows, with
compression), fold64 (the fp64 server-side folds) and mewma64 (the CFA-GE update, rows updated
in place). Reference rules: TF2 consensus_v3.py:153-155, TF1 cfa.py:69-76,
cfa_ongraphs.py:225-273, cfa_ge_2stage.py:594-606, parameter_server_v2.py:159-161.
"""
import numpy as np
import pytest

from oracle import cfa_oracle as O

pytestmark = pytest.mark.gpu

SHAPES = [(1024, 1024), (1024,), (1024, 2048), (2048,)]  # P = 3 148 800 elements
CALLS = 3


def _model(rng, dtype=np.float32, scale=1.0):
    return [(rng.standard_normal(s) * scale).astype(dtype) for s in SHAPES]


@pytest.fixture
def R(monkeypatch):
    from federated_amd.consensus import _runtime as R
    monkeypatch.setattr(R, "SIGNAL_COMPLETION", True)
    monkeypatch.setattr(R, "SIGNAL_SPIN_US", 2000000)  # a large P: the word, not the fallback, ends the wait
    return R


def _staged(R, monkeypatch, fn):
    """fn() on the staged path (no zero-copy rows, no completion word)."""
    with monkeypatch.context() as m:
        m.setattr(R, "SINGLE_ZERO_COPY", False)
        m.setattr(R, "TF1_ZERO_COPY", False)
        m.setattr(R, "SIGNAL_COMPLETION", False)
        return fn()


def _equal(got, want):
    assert len(got) == len(want)
    for k, (g, w) in enumerate(zip(got, want)):
        g, w = np.asarray(g), np.asarray(w)
        assert g.dtype == w.dtype and g.size == w.size, k
        assert np.array_equal(g.reshape(-1), w.reshape(-1)), k


def test_f32_compression_kind(R, monkeypatch):
    rng = np.random.default_rng(4200)
    mx = R.mixer()
    al = [0.25, 0.25, 0.25]
    for call in range(CALLS):
        local, nbrs = _model(rng, scale=1e-3), [_model(rng, scale=1e-3) for _ in range(3)]
        got, kept = mx.mix(local, nbrs, al, compress=(2, 2))
        want, want_kept = _staged(R, monkeypatch, lambda: mx.mix(local, nbrs, al, compress=(2, 2)))
        _equal(got, want)
        assert kept == want_kept, call
        # the first layers (no epilogue) are the oracle's sequential mix
        ref = O.sequential_mix(local[0].reshape(-1), [x[0].reshape(-1) for x in nbrs], al)
        assert np.array_equal(np.asarray(got[0]).reshape(-1), ref), call


def test_f32_tf1_rule_kind(R, monkeypatch):
    rng = np.random.default_rng(4201)
    mx = R.mixer()
    al = [float(np.float64(0.5) * np.float64(1 / 3)), float(np.float64(0.5) * np.float64(0.25))]
    for call in range(CALLS):
        local, nbrs = _model(rng), [_model(rng) for _ in range(2)]
        got, _ = mx.mix(local, nbrs, al, tf1=True)
        want, _ = _staged(R, monkeypatch, lambda: mx.mix(local, nbrs, al, tf1=True))
        _equal(got, want)
        ref = O.tf1_mix_flat(local[2].reshape(-1), [x[2].reshape(-1) for x in nbrs], al)
        assert np.array_equal(np.asarray(got[2]).reshape(-1), ref.astype(np.float32)), call


def test_tf1w_kind(R, monkeypatch):
    rng = np.random.default_rng(4202)
    mx = R.mixer()
    al = [0.2, 0.15, 0.1]
    for call in range(CALLS):
        local, nbrs = _model(rng, scale=1e-3), [_model(rng, scale=1e-3) for _ in range(3)]
        got, kept = mx.mix_tf1(local, nbrs, al, compress=(3, 2))
        want, want_kept = _staged(R, monkeypatch, lambda: mx.mix_tf1(local, nbrs, al, compress=(3, 2)))
        _equal(got, want)
        assert kept == want_kept, call
        ref = O.tf1_mix_flat(local[0].reshape(-1), [x[0].reshape(-1) for x in nbrs], al)
        assert np.array_equal(np.asarray(got[0]).reshape(-1), ref), call


def test_f64_kind(R, monkeypatch):
    rng = np.random.default_rng(4203)
    mx = R.mixer()
    al = [0.2, 0.15]
    for call in range(CALLS):
        local = _model(rng, np.float64, 1e-3)
        nbrs = [_model(rng, np.float64, 1e-3) for _ in range(2)]
        got, kept = mx.mix_tf1(local, nbrs, al, compress=(1, 2))
        want, want_kept = _staged(R, monkeypatch, lambda: mx.mix_tf1(local, nbrs, al, compress=(1, 2)))
        _equal(got, want)
        assert kept == want_kept, call
        ref = O.tf1_mix_flat(local[3], [x[3] for x in nbrs], al)
        assert np.array_equal(np.asarray(got[3]).reshape(-1), ref), call


@pytest.mark.parametrize("rule", [0, 3])
def test_fold64_kind(R, monkeypatch, rule):
    from federated_amd import _lib
    rng = np.random.default_rng(4204 + rule)
    mx = R.mixer()
    n = 4
    al = [0.9] * n
    div = [float(n)] * n if rule == _lib.RULE_SEQUENTIAL_DIV else None
    for call in range(CALLS):
        local = _model(rng, np.float64)
        nbrs = [_model(rng, np.float64) for _ in range(n)]
        got = mx.fold64(local, nbrs, al, rule, div)
        want = _staged(R, monkeypatch, lambda: mx.fold64(local, nbrs, al, rule, div))
        _equal(got, want)


def test_mewma64_kind(R, monkeypatch):
    rng = np.random.default_rng(4206)
    mx = R.mixer()
    N, n = 3, 2
    for call in range(CALLS):
        W = _model(rng, np.float64)
        grads = [_model(rng, np.float64) for _ in range(n)]
        states = [rng.standard_normal(s + (N,)) for s in SHAPES]
        states_staged = [s.copy() for s in states]
        got = mx.mewma_tf1(W, states, grads, 0.99, (0.1, 0.1, 0.2, 0.2), False, True)
        want = _staged(R, monkeypatch,
                       lambda: mx.mewma_tf1(W, states_staged, grads, 0.99, (0.1, 0.1, 0.2, 0.2), False, True))
        _equal(got, want)
        for k in range(len(SHAPES)):
            assert np.array_equal(states[k], states_staged[k]), (call, k)
