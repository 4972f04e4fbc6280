"""The division rule of the fp32 divisor fold (cfa_internal.h div_rd, used by cfa_mix_seq_div_f32
for the FedAvg step p + u*(x - p)/C, parameter_server_v2.py:159-161): (float)((double)a *
RN_64(1/(double)C)) must be IEEE fp32 a / C for every fp32 a and C whose quotient is not subnormal;
a subnormal quotient (0 < |p| < 2^-126) takes the IEEE division instead, because it can sit exactly
on a rounding midpoint (round-4 advisor finding). This checks the arithmetic claim itself on the CPU (numpy's fp64 multiply and fp64 -> fp32 conversion round as the GPU's
v_mul_f64 / v_cvt_f32_f64 do), over random bit patterns of both operands and the IEEE specials;
the GPU test test_mix_seq_div_quotient_exact_over_exponent_range checks the kernel."""
import numpy as np
import pytest


def _one_multiply(a, c):
    return (a.astype(np.float64) * (1.0 / c.astype(np.float64))).astype(np.float32)


def _div_rd(a, c):
    """cfa_internal.h div_rd: the one-multiply form, the IEEE division where 0 < |p| < 2^-126."""
    p = a.astype(np.float64) * (1.0 / c.astype(np.float64))
    m = np.abs(p)
    slow = (m < 2.0 ** -126) & (m != 0)
    return np.where(slow, a / c, p.astype(np.float32))


def subnormal_ties(n_odd=4096, o_max=2000):
    """(a, C) with a / C exactly on a subnormal rounding midpoint: a = k * o * 2^-149 (k odd, k * o
    < 2^24 so a is exact), C = 2 o, quotient (k o / 2o) * 2^-149 = (k / 2) * 2^-149."""
    aa, cc = [], []
    k = np.arange(1, n_odd * 2, 2, dtype=np.float64)
    for o in range(1, o_max, 2):
        kk = k[k * o < 2 ** 24]
        aa.append((kk * o * 2.0 ** -149).astype(np.float32))
        cc.append(np.full(kk.size, 2 * o, np.float32))
    return np.concatenate(aa), np.concatenate(cc)


def _same(got, ref):
    return (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))


@pytest.mark.parametrize("seed", range(4))
def test_random_bit_patterns(seed):
    rng = np.random.default_rng(9100 + seed)
    n = 2_000_000
    a = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    c = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    with np.errstate(all="ignore"):
        ok = _same(_div_rd(a, c), a / c)
    assert ok.all(), (a[~ok][:4], c[~ok][:4])


def test_specials_and_near_midpoint_quotients():
    fi = np.finfo(np.float32)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, fi.smallest_subnormal, -fi.smallest_subnormal,
                   fi.smallest_normal, fi.max, -fi.max, 1.0, 3.0, 7.0, 0.1, 1e-40, 2.0 ** -126, 2.0 ** 127],
                  dtype=np.float32)
    a, c = np.meshgrid(sp, sp)
    a, c = a.ravel(), c.ravel()
    # quotients whose exact value sits close to a rounding midpoint: a = (2k + 1) * C / 2 rounded
    rng = np.random.default_rng(9199)
    k = rng.integers(1 << 22, 1 << 23, 500_000).astype(np.float64)
    cc = rng.integers(3, 1 << 24, k.size).astype(np.float64)
    aa = ((2 * k + 1) * cc / 2).astype(np.float32)
    a = np.concatenate([a, aa])
    c = np.concatenate([c, cc.astype(np.float32)])
    with np.errstate(all="ignore"):
        ok = _same(_div_rd(a, c), a / c)
    assert ok.all(), (a[~ok][:4], c[~ok][:4])


def test_exact_subnormal_ties():
    """The one-multiply form alone rounds some exact subnormal midpoints the wrong way (e.g.
    a = 147 * 2^-149, C = 98: 1 ulp instead of ties-to-even's 2); the guarded rule does not."""
    a, c = subnormal_ties()
    with np.errstate(all="ignore"):
        ref = a / c
        assert not _same(_one_multiply(a, c), ref).all()  # the finding this guards against
        ok = _same(_div_rd(a, c), ref)
        neg = _same(_div_rd(-a, c), -a / c)
    assert ok.all() and neg.all(), (a[~ok][:4], c[~ok][:4])
