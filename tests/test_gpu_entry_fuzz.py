"""Randomised parity of every streaming entry point against numpy, through the C-ABI.

The kernel tests pin each entry point at chosen sizes; this draws the shape of every call at
random, so the pieces a kernel splits a call into (scalar head for a misaligned view, full
tiles, the partial tile, the scalar tail, passes chained above CFA_MAX_FANIN, the launch-shape
bands by size) meet in combinations no hand-written case lists:

- P from 0 to ~3M (log-uniform, plus tiny sizes), every buffer a view at its own element
  offset 0..3 (same offsets: head + vector body; mixed: the scalar path);
- n from 0 to 20 (sometimes up to 40: chained passes), coefficients 1/(n+1), uniform in (0, 1]
  or outside it (negative, > 1), in place (out = local) or not;
- compression modes 0..4 on a random range, for the fused and the standalone epilogues.

Bars (the same as the kernel tests): bit-exact against the numpy restatement of the reference
rule (NaN matches NaN), counts exact. References: TF2 consensus_v3.py:153-155 (sequential),
parameter_server_v2.py:159-161 (divisor fold), cfa_ongraphs.py:225-273 (compression), TF1
cfa.py:69-76 (TF1 chain), cfa_ge_2stage.py:591-621 (MEWMA).

CFA_FUZZ_CASES (default 80) sets the number of cases; CFA_FUZZ_SEED the first seed.
"""
import os

import numpy as np
import pytest
import torch

from oracle import cfa_oracle as O

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("CFA_FUZZ_CASES", "80"))
SEED0 = int(os.environ.get("CFA_FUZZ_SEED", "52000"))
KINDS = ["seq", "div", "seq_compress", "compress", "tf1", "tf1_wide", "tf1_f64", "fold_f64", "mewma", "mewma_f64"]


def _size(rng):
    r = rng.random()
    if r < 0.15:
        return int(rng.integers(0, 40))
    if r < 0.3:
        return int(rng.integers(40, 5000))
    return int(np.exp(rng.uniform(np.log(5000), np.log(3_200_000))))


def _view(host, off):
    """A device view of ``host`` starting ``off`` elements into a larger allocation."""
    base = torch.zeros(host.size + 4, dtype=torch.float32 if host.dtype == np.float32 else torch.float64,
                       device="cuda")
    v = base[off:off + host.size]
    if host.size:
        v.copy_(torch.from_numpy(host))
    return v


def _alphas(rng, n):
    r = rng.random()
    if r < 0.4:
        return [1.0 / (n + 1)] * n
    if r < 0.85:
        return [float(v) for v in rng.uniform(1e-3, 1.0, n)]
    return [float(v) for v in rng.uniform(-1.5, 2.5, n)]


def _same(got, ref):
    got, ref = np.asarray(got), np.asarray(ref)
    if got.shape != ref.shape:
        return False
    iv = np.uint32 if got.dtype == np.float32 else np.uint64
    return bool(np.all((got.view(iv) == ref.astype(got.dtype).view(iv)) | (np.isnan(got) & np.isnan(ref))))


def _offsets(rng, k):
    if rng.random() < 0.6:
        o = int(rng.integers(0, 4)) if rng.random() < 0.5 else 0
        return [o] * k
    return [int(v) for v in rng.integers(0, 4, k)]


def _crange(rng, P):
    if P == 0:
        return 0, 0
    a = int(rng.integers(0, P + 1))
    b = int(rng.integers(a, P + 1))
    return a, b


@pytest.mark.parametrize("case", range(CASES))
def test_entry_point_fuzz(gpu, case):
    rng = np.random.default_rng(SEED0 + case)
    kind = KINDS[case % len(KINDS)]
    P = _size(rng)
    n = int(rng.integers(0, 21)) if rng.random() < 0.9 else int(rng.integers(17, 41))
    f64 = kind in ("tf1_f64", "fold_f64", "mewma_f64")
    dt = np.float64 if f64 else np.float32
    scale = 10.0 ** rng.uniform(-3, 1)
    rnd = lambda: (rng.standard_normal(P) * scale).astype(dt)
    info = (kind, P, n)

    if kind in ("seq", "div", "seq_compress"):
        if kind == "seq_compress":
            n = min(n, 16)  # the fused epilogue takes one pass of at most CFA_MAX_FANIN
        local, nbrs = rnd(), [rnd() for _ in range(n)]
        al = _alphas(rng, n)
        offs = _offsets(rng, n + 2)
        inplace = rng.random() < 0.3
        dl = _view(local, offs[0])
        out = dl if inplace else _view(np.zeros(P, np.float32), offs[1])
        dn = [_view(x, o) for x, o in zip(nbrs, offs[2:])]
        if kind == "seq":
            ref = O.sequential_mix(local, nbrs, al)
            gpu.mix_seq(out, dl, dn, al)
        elif kind == "div":
            dv = [float(v) for v in rng.integers(1, 33, n)] if rng.random() < 0.7 else \
                [float(v) for v in rng.uniform(0.05, 50.0, n)]
            ref = local.copy()
            for x, a, d in zip(nbrs, al, dv):
                ref = ref + np.float32(a) * (x - ref) / np.float32(d)
            gpu.mix_seq_div(out, dl, dn, al, dv)
        else:
            mode = int(rng.integers(0, 5))
            cb, ce = _crange(rng, P)
            y = O.sequential_mix(local, nbrs, al).astype(np.float32).copy()
            seg = y[cb:ce].reshape(1, -1)
            cnt = O.tf1_compress(seg, local[cb:ce].reshape(1, -1), mode) if mode else ce - cb
            y[cb:ce] = seg.reshape(-1)
            ref = y
            kept = torch.zeros(1, dtype=torch.int64, device="cuda")
            gpu.mix_seq_compress(out, dl, dn, al, mode, cb, ce, kept)
            assert int(kept.item()) == cnt, info
        assert _same(out.cpu().numpy(), ref), info + (offs, inplace)
        return

    if kind == "compress":
        mode = int(rng.integers(1, 5))
        ref_b = (rng.standard_normal(P) * 1e-2).astype(np.float32)
        y = (ref_b + (rng.standard_normal(P) * 2e-3).astype(np.float32)) if mode in (2, 3) else \
            (rng.standard_normal(P) * 1e-2).astype(np.float32)
        expect = y.copy().reshape(1, -1)
        cnt = O.tf1_compress(expect, (ref_b if mode in (2, 3) else y).reshape(1, -1), mode)
        offs = _offsets(rng, 2)
        dy = _view(y, offs[0])
        kept = torch.zeros(1, dtype=torch.int64, device="cuda")
        gpu.compress(dy, _view(ref_b, offs[1]) if mode in (2, 3) else None, mode, kept)
        assert _same(dy.cpu().numpy(), expect.reshape(-1)), info + (offs, mode)
        assert int(kept.item()) == cnt, info
        return

    if kind in ("tf1", "tf1_wide"):
        if kind == "tf1_wide":
            n = max(n, 1)
        local, nbrs = rnd(), [rnd() for _ in range(n)]
        al = [float(a) for a in _alphas(rng, n)]
        mode = int(rng.integers(0, 5)) if rng.random() < 0.5 else 0
        cb, ce = _crange(rng, P) if mode else (0, 0)
        y = O.tf1_mix_flat(local, nbrs, al)
        y = y.astype(np.float64) if n else y.astype(np.float32).copy()
        cnt = None
        if mode:
            seg = y[cb:ce].reshape(1, -1)
            cnt = O.tf1_compress(seg, local[cb:ce].reshape(1, -1), mode)
            y[cb:ce] = seg.reshape(-1)
        offs = _offsets(rng, n + 1)
        dl = _view(local, offs[0])
        dn = [_view(x, o) for x, o in zip(nbrs, offs[1:])]
        kept = torch.zeros(1, dtype=torch.int64, device="cuda") if mode else None
        if kind == "tf1":
            out = _view(np.zeros(P, np.float32), int(rng.integers(0, 4)))
            gpu.mix_tf1(out, dl, dn, al, mode, cb, ce, kept)
            assert _same(out.cpu().numpy(), y.astype(np.float32)), info + (offs, mode)
        else:
            from federated_amd import _lib
            o64 = _view(np.zeros(P, np.float64), int(rng.integers(0, 4)))
            _lib.call("cfa_mix_tf1_wide_f32", o64.data_ptr(), dl.data_ptr(),
                      _lib.ptr_table([x.data_ptr() for x in dn]), _lib.double_array(al), n, P, mode, cb, ce,
                      kept.data_ptr() if kept is not None else None, gpu.stream_handle())
            assert _same(o64.cpu().numpy(), y.astype(np.float64)), info + (offs, mode)
        if mode:
            assert int(kept.item()) == cnt, info
        return

    if kind == "tf1_f64":
        n = max(n, 1)
        local, nbrs = rnd(), [rnd() for _ in range(n)]
        al = [float(a) for a in _alphas(rng, n)]
        ref = O.tf1_mix_flat(local, nbrs, al)
        offs = _offsets(rng, n + 2)
        out = _view(np.zeros(P, np.float64), offs[1])
        gpu.mix_tf1_f64(out, _view(local, offs[0]), [_view(x, o) for x, o in zip(nbrs, offs[2:])], al, False)
        assert _same(out.cpu().numpy(), ref), info + (offs,)
        return

    if kind == "fold_f64":
        rule = int(rng.choice([0, 2, 3]))
        local, nbrs = rnd(), [rnd() for _ in range(n)]
        al = [float(a) for a in _alphas(rng, n)]
        dv = [float(v) for v in rng.integers(1, 33, n)]
        ref = local.copy()
        for j in range(n):
            if rule == 0:
                ref = ref + al[j] * (nbrs[j] - ref)
            elif rule == 2:
                ref = ref + al[j] * (nbrs[j] - ref) / dv[j]
            else:
                ref = ref + al[j] * nbrs[j]
        offs = _offsets(rng, n + 2)
        out = _view(np.zeros(P, np.float64), offs[1])
        gpu.fold_f64(out, _view(local, offs[0]), [_view(x, o) for x, o in zip(nbrs, offs[2:])], al, rule,
                     dv if rule == 2 else None)
        assert _same(out.cpu().numpy(), ref), info + (offs, rule)
        return

    # MEWMA (fp32 buckets: cfa_mewma_update_f32; fp64: cfa_mewma_tf1_f64, all-fp64 arrays)
    n = max(1, min(n, 8))
    rho = float(rng.choice([0.99, 0.9, 0.5]))
    lr1, lr2 = float(rng.uniform(1e-3, 0.2)), float(rng.uniform(1e-3, 0.2))
    split = int(rng.integers(0, P + 1)) if P else 0
    init, filtered = bool(rng.random() < 0.3), bool(rng.random() < 0.5)
    W, s, g = rnd(), [rnd() for _ in range(n)], [rnd() for _ in range(n)]
    offs = _offsets(rng, 2 * n + 1)
    dW = _view(W, offs[0])
    ds = [_view(x, o) for x, o in zip(s, offs[1:n + 1])]
    dg = [_view(x, o) for x, o in zip(g, offs[n + 1:])]
    Wr, sr = W.copy(), [x.copy() for x in s]
    if kind == "mewma":
        lr = np.where(np.arange(P) < split, np.float32(lr1), np.float32(lr2)).astype(np.float32)
        for j in range(n):
            sr[j] = g[j].copy() if init else rho * g[j] + (1 - rho) * sr[j]
            Wr = Wr - lr * (sr[j] if filtered else g[j])
        gpu.mewma(dW, ds, dg, rho, lr1, lr2, split, init, filtered)
    else:
        lr = np.where(np.arange(P) < split, lr1, lr2)
        for j in range(n):
            sr[j] = g[j].copy() if init else rho * g[j] + (1 - rho) * sr[j]
            Wr = Wr - lr * (sr[j] if filtered else g[j])
        gpu.mewma_tf1_f64(dW, ds, dg, rho, lr1, lr2, split, init, filtered, 0)
    assert _same(dW.cpu().numpy(), Wr), info + (offs, init, filtered)
    for j in range(n):
        assert _same(ds[j].cpu().numpy(), sr[j]), info + (j, offs)
