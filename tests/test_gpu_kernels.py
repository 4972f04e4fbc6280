"""GPU parity of the libcfa kernels against the CPU oracle, called through the C-ABI.

Bars: the sequential rule is bit-exact against fp32 numpy (same three roundings);
the TF1 rule (cfa_mix_tf1_f32) is bit-exact against the fp64 reference chain rounded once to
fp32; the linear closed form is within 1e-5 normwise (max|y - r| <= 1e-5 * max|r|);
compression counts are exact integers."""
import numpy as np
import pytest
import torch

from conftest import normwise_close
from oracle import cfa_oracle as O

pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _rand(rng, n, P, scale=1.0):
    return [(rng.standard_normal(P) * scale).astype(np.float32) for _ in range(n)]


SIZES = [0, 1, 3, 4, 5, 255, 1023, 4096 + 3, 1 << 20, 3 * (1 << 20) + 7]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 8, 16, 17, 33])
def test_mix_seq_bitexact(gpu, n):
    rng = np.random.default_rng(100 + n)
    for P in SIZES:
        local = _rand(rng, 1, P)[0]
        nbrs = _rand(rng, n, P)
        alphas = [1.0 / (n + 1)] * n if n else []
        ref = O.sequential_mix(local, nbrs, alphas)
        out = torch.empty(P, dtype=torch.float32, device="cuda")
        gpu.mix_seq(out, _dev(local), [_dev(x) for x in nbrs], alphas)
        assert np.array_equal(out.cpu().numpy(), ref), (n, P)


@pytest.mark.parametrize("n", [2, 4, 8, 12, 16, 20])
def test_mix_seq_bitexact_across_launch_shape_bands(gpu, n):
    """The default launch shape depends on the bucket size (cfa_internal.h mix_auto_shape): one
    workgroup per CU from 8M elements, four below (1 float4 per lane from 512K, 4 from 1.5M, 2 for
    more than 9 neighbours up to 3M). Sizes on both sides of every band edge, with ragged tails."""
    rng = np.random.default_rng(300 + n)
    for P in [524_287, 524_293, 1_572_861, 1_572_873, 2_000_003, 3_145_731, 3_145_741, 8_388_607,
              8_388_613]:
        local = _rand(rng, 1, P)[0]
        nbrs = _rand(rng, n, P)
        alphas = [1.0 / (n + 1)] * n
        ref = O.sequential_mix(local, nbrs, alphas)
        out = torch.empty(P, dtype=torch.float32, device="cuda")
        gpu.mix_seq(out, _dev(local), [_dev(x) for x in nbrs], alphas)
        assert np.array_equal(out.cpu().numpy(), ref), (n, P)


@pytest.mark.parametrize("n", [2, 8, 12, 20])
def test_mix_seq_div_bitexact_across_launch_shape_bands(gpu, n):
    """The divisor fold takes the mix's shape bands since round 4, with four float4 per lane (two
    above nine neighbours) in the one-workgroup band from 8M elements: sizes on both sides of the
    band edges, ragged tails, a divisor that is not a power of two, u != 1, in place at 8M+."""
    rng = np.random.default_rng(320 + n)
    for P in [524_293, 1_572_873, 3_145_741, 8_388_607, 8_388_613, 9_000_005]:
        local = _rand(rng, 1, P)[0]
        nbrs = _rand(rng, n, P)
        w = local.copy()  # parameter_server_v2.py:159-161 with u = 0.99, C = 7 (fp32 numpy)
        for x in nbrs:
            w = w + np.float32(0.99) * (x - w) / np.float32(7.0)
        inplace = P > 8_388_608
        out = _dev(local) if inplace else torch.empty(P, dtype=torch.float32, device="cuda")
        gpu.mix_seq_div(out, out if inplace else _dev(local), [_dev(x) for x in nbrs], [0.99] * n, [7.0] * n)
        assert np.array_equal(out.cpu().numpy(), w), (n, P)


def test_mix_seq_varied_alphas_and_inplace(gpu):
    rng = np.random.default_rng(7)
    P = 1_000_003
    local = _rand(rng, 1, P)[0]
    nbrs = _rand(rng, 5, P)
    alphas = [0.1, 0.5, 1.0, 0.3333333, 0.9]
    ref = O.sequential_mix(local, nbrs, alphas)
    w = _dev(local)
    gpu.mix_seq(w, w, [_dev(x) for x in nbrs], alphas)  # out aliases local
    assert np.array_equal(w.cpu().numpy(), ref)


@pytest.mark.parametrize("offsets", [(1, 1, 1), (2, 2, 2), (3, 3, 3), (0, 1, 2), (1, 0, 3)])
def test_mix_seq_misaligned_views(gpu, offsets):
    """Sub-tensor views at element offsets: same misalignment -> scalar head + float4 body,
    mixed misalignment -> scalar path. Results identical either way."""
    rng = np.random.default_rng(11)
    P = 100_003
    base = [_dev(np.zeros(P + 8, np.float32)) for _ in range(3)]
    local = _rand(rng, 1, P)[0]
    nbrs = _rand(rng, 2, P)
    o_out, o_loc, o_nb = offsets
    out = base[0][o_out:o_out + P]
    loc = base[1][o_loc:o_loc + P]
    loc.copy_(_dev(local))
    nb0 = base[2][o_nb:o_nb + P]
    nb0.copy_(_dev(nbrs[0]))
    gpu.mix_seq(out, loc, [nb0, _dev(nbrs[1])], [1 / 3, 1 / 3])
    assert np.array_equal(out.cpu().numpy(), O.sequential_mix(local, nbrs, [1 / 3, 1 / 3]))


@pytest.mark.parametrize("n", [1, 3, 8, 20])
def test_mix_linear_closed_form(gpu, n):
    rng = np.random.default_rng(200 + n)
    P = 2_000_001
    local = _rand(rng, 1, P)[0]
    nbrs = _rand(rng, n, P)
    alphas = [1.0 / (n + 1)] * n
    coeff = O.closed_form_coeffs(alphas)
    out = torch.empty(P, dtype=torch.float32, device="cuda")
    gpu.mix_linear(out, _dev(local), [_dev(x) for x in nbrs], coeff)
    ref = O.sequential_mix(local.astype(np.float64), [x.astype(np.float64) for x in nbrs], alphas)
    assert normwise_close(out.cpu().numpy(), ref)


def _compress_expect(local, nbrs, alphas, mode, cb, ce):
    """fp32 chain, then the epilogue as numpy 2 evaluates it on fp32 arrays (threshold and
    replacement cast to fp32; W2 is [4096, 6])."""
    y = O.sequential_mix(local, nbrs, alphas).astype(np.float32).copy()
    seg = y[cb:ce].reshape(-1, 6)
    cnt = O.tf1_compress(seg, local[cb:ce].reshape(-1, 6), mode)
    y[cb:ce] = seg.reshape(-1)
    return y, cnt


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
def test_compress_fp32_threshold_boundaries(gpu, mode):
    """fp32(0.01) < 0.01 and fp32(1e-4) < 1e-4 in exact arithmetic, but numpy 2 compares an fp32
    array with a Python float in fp32: the boundary values are kept, not replaced."""
    thr = {1: 1e-3, 2: 1e-4, 3: 1e-3, 4: 1e-2}[mode]
    t32 = np.float32(thr)
    edge = np.array([t32, -t32, np.nextafter(t32, np.float32(0)), -np.nextafter(t32, np.float32(0)),
                     np.nextafter(t32, np.float32(1)), 0.0, -0.0, 5e-5, -5e-5, 0.5] * 6, dtype=np.float32)
    ref = (np.arange(edge.size, dtype=np.float32) * np.float32(1e-3)) if mode in (2, 3) else None
    y = edge + ref if ref is not None else edge.copy()
    expect = y.copy().reshape(-1, 6)
    cnt = O.tf1_compress(expect, (ref if ref is not None else y).reshape(-1, 6), mode)
    dy = _dev(y)
    kept = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu.compress(dy, _dev(ref) if ref is not None else None, mode, kept)
    assert np.array_equal(dy.cpu().numpy(), expect.reshape(-1)), mode
    assert int(kept.item()) == cnt


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
def test_compress_epilogue_grid_stride_large(gpu, mode):
    """The standalone epilogue at more full tiles than the grid has workgroups (each walks several,
    the partial tile by one workgroup), an odd P (scalar tail), values around every threshold:
    identical to numpy, count included (round 4 skeleton, compile-time mode form)."""
    rng = np.random.default_rng(330 + mode)
    P = 4_000_003
    ref = (rng.standard_normal(P) * 1e-2).astype(np.float32)
    y = (ref + rng.standard_normal(P).astype(np.float32) * np.float32(2e-3)) if mode in (2, 3) else \
        (rng.standard_normal(P) * 1e-2).astype(np.float32)
    expect = y.copy().reshape(1, -1)
    cnt = O.tf1_compress(expect, (ref if mode in (2, 3) else y).reshape(1, -1), mode)
    if mode == 0:
        cnt = P  # no epilogue: every element kept
    dy = _dev(y)
    kept = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu.compress(dy, _dev(ref) if mode in (2, 3) else None, mode, kept)
    assert np.array_equal(dy.cpu().numpy(), expect.reshape(-1))
    assert int(kept.item()) == cnt


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("n", [0, 1, 3, 17])
def test_mix_seq_compress(gpu, mode, n):
    rng = np.random.default_rng(300 + 10 * mode + n)
    P = 24_622  # FL_CFA_CNN_tf2 bucket; W2 = [40, 24616)
    cb, ce = 40, 40 + 24_576
    base = (rng.standard_normal(P) * 0.01).astype(np.float32)
    local = base + (rng.standard_normal(P) * 3e-4).astype(np.float32)
    nbrs = [base + (rng.standard_normal(P) * 3e-4).astype(np.float32) for _ in range(n)]
    alphas = [1.0 / (n + 1)] * n
    ref, cnt = _compress_expect(local, nbrs, alphas, mode, cb, ce)
    out = torch.empty(P, dtype=torch.float32, device="cuda")
    kept = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu.mix_seq_compress(out, _dev(local), [_dev(x) for x in nbrs], alphas, mode, cb, ce, kept)
    assert np.array_equal(out.cpu().numpy(), ref)
    assert int(kept.item()) == cnt
    if mode in (1, 2, 4) and (n or mode in (1, 4)):
        assert 0 < cnt < ce - cb  # the regime exercises both branches
    elif mode in (2, 3) and not n:
        assert cnt == 0  # DPCM with no neighbour: y == ref everywhere (cfa_ongraphs.py:218-249)


# ---- TF1 numerics (cfa_mix_tf1_f32): fp64 chain, one rounding; bit-exact vs fp32(reference) ----
def _tf1_alphas(n, eps=0.7, devices=8):
    return [eps * O.tf1_weight_factor(devices, 1, j % devices, max(n - 1, 0)) for j in range(n)]


@pytest.mark.parametrize("n", [1, 2, 3, 8, 16, 17, 33])
def test_mix_tf1_bitexact(gpu, n):
    rng = np.random.default_rng(700 + n)
    alphas = _tf1_alphas(n)
    for P in [1, 3, 4, 5, 1023, 24_622, 1 << 20]:
        local = _rand(rng, 1, P)[0]
        nbrs = _rand(rng, n, P)
        ref = O.tf1_mix_flat(local, nbrs, alphas)
        assert ref.dtype == np.float64
        out = torch.empty(P, dtype=torch.float32, device="cuda")
        gpu.mix_tf1(out, _dev(local), [_dev(x) for x in nbrs], alphas)
        assert np.array_equal(out.cpu().numpy(), ref.astype(np.float32)), (n, P)


@pytest.mark.parametrize("offsets", [(1, 1, 1), (3, 3, 3), (0, 1, 2)])
def test_mix_tf1_misaligned_and_inplace(gpu, offsets):
    rng = np.random.default_rng(17)
    P, n = 50_001, 3
    alphas = _tf1_alphas(n, 1.0)
    local = _rand(rng, 1, P)[0]
    nbrs = _rand(rng, n, P)
    ref = O.tf1_mix_flat(local, nbrs, alphas).astype(np.float32)
    base = [_dev(np.zeros(P + 8, np.float32)) for _ in range(2)]
    o_out, o_loc, o_nb = offsets
    out, loc = base[0][o_out:o_out + P], base[1][o_loc:o_loc + P]
    loc.copy_(_dev(local))
    nb0 = _dev(np.zeros(P + 8, np.float32))[o_nb:o_nb + P]
    nb0.copy_(_dev(nbrs[0]))
    gpu.mix_tf1(out, loc, [nb0] + [_dev(x) for x in nbrs[1:]], alphas)
    assert np.array_equal(out.cpu().numpy(), ref)
    w = _dev(local)
    gpu.mix_tf1(w, w, [_dev(x) for x in nbrs], alphas)  # out aliases local
    assert np.array_equal(w.cpu().numpy(), ref)


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("n", [0, 1, 3, 17])
def test_mix_tf1_compress(gpu, mode, n):
    """Fused fp64 epilogue: the reference compresses its fp64 W_up_l2 against the fp32 n_W_l2
    (cfa_ongraphs.py:225-273); the test and replacement in fp64, the count exact."""
    rng = np.random.default_rng(900 + 10 * mode + n)
    P = 24_622
    cb, ce = 40, 40 + 24_576
    base = (rng.standard_normal(P) * 0.01).astype(np.float32)
    local = base + (rng.standard_normal(P) * 3e-4).astype(np.float32)
    nbrs = [base + (rng.standard_normal(P) * 3e-4).astype(np.float32) for _ in range(n)]
    alphas = [0.9 / (n + 1) * 2] * n
    y = O.tf1_mix_flat(local, nbrs, alphas)
    y = y.astype(np.float64) if n else y.copy()
    seg = y[cb:ce].reshape(-1, 6)
    cnt = O.tf1_compress(seg, local[cb:ce].reshape(-1, 6), mode)
    y[cb:ce] = seg.reshape(-1)
    out = torch.empty(P, dtype=torch.float32, device="cuda")
    kept = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu.mix_tf1(out, _dev(local), [_dev(x) for x in nbrs], alphas, mode, cb, ce, kept)
    assert np.array_equal(out.cpu().numpy(), y.astype(np.float32)), (mode, n)
    assert int(kept.item()) == cnt  # mode 0: the whole range (counter_param = W2 size)
    if mode in (1, 2, 4) and (n or mode in (1, 4)):
        assert 0 < cnt < ce - cb


# ---- fp64 buckets (cfa_mix_tf1_f64 / cfa_mewma_tf1_f64): the reference's dtypes and values ----
def _dev64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()


@pytest.mark.parametrize("n", [1, 2, 5, 16, 17, 40])
@pytest.mark.parametrize("dtypes", ["f32", "f64", "local64"])
def test_mix_tf1_f64_identical(gpu, n, dtypes):
    """Any mix of fp32/fp64 reference arrays: identical to numpy's result, dtype included."""
    rng = np.random.default_rng(1100 + n)
    P = 30_011
    alphas = _tf1_alphas(n)
    local = _rand(rng, 1, P)[0]
    nbrs = _rand(rng, n, P)
    if dtypes == "f64":
        local, nbrs = rng.standard_normal(P), [rng.standard_normal(P) for _ in range(n)]
    elif dtypes == "local64":
        local = local.astype(np.float64) * (1 + 1e-9)
    ref = O.tf1_mix_flat(local, nbrs, alphas)
    assert ref.dtype == np.float64
    out = torch.empty(P, dtype=torch.float64, device="cuda")
    step0_f32 = local.dtype == np.float32 and nbrs[0].dtype == np.float32
    gpu.mix_tf1_f64(out, _dev64(local), [_dev64(x) for x in nbrs], alphas, step0_f32)
    assert np.array_equal(out.cpu().numpy(), ref), (n, dtypes)


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
def test_mix_tf1_f64_compress(gpu, mode):
    rng = np.random.default_rng(1200 + mode)
    P, n = 24_622, 3
    cb, ce = 40, 40 + 24_576
    base = (rng.standard_normal(P) * 0.01).astype(np.float32)
    local = base + (rng.standard_normal(P) * 3e-4).astype(np.float32)
    nbrs = [base + (rng.standard_normal(P) * 3e-4).astype(np.float32) for _ in range(n)]
    alphas = [0.45] * n
    y = O.tf1_mix_flat(local, nbrs, alphas)
    seg = y[cb:ce].reshape(-1, 6)
    cnt = O.tf1_compress(seg, local[cb:ce].reshape(-1, 6), mode)
    y[cb:ce] = seg.reshape(-1)
    out = torch.empty(P, dtype=torch.float64, device="cuda")
    kept = torch.zeros(1, dtype=torch.int64, device="cuda")
    gpu.mix_tf1_f64(out, _dev64(local), [_dev64(x) for x in nbrs], alphas, True, mode, cb, ce, kept)
    assert np.array_equal(out.cpu().numpy(), y)
    assert int(kept.item()) == cnt


@pytest.mark.parametrize("filtered,init", [(True, False), (False, False), (False, True)])
@pytest.mark.parametrize("dtypes", ["s64_g64_w64", "s32_g64_w64", "s64_g32_w64", "s32_g32_w32", "s32_g32_w64"])
def test_mewma_tf1_f64_identical(gpu, filtered, init, dtypes):
    """cfa_ge_2stage.py:331-371 / :593-621 on the reference's arrays, every dtype combination
    numpy 2 can meet: the driver's fp64 saved states (np.zeros) and fp64 datagrad gradients, and
    fp32 variants of each; the result equals numpy's, dtype included."""
    from federated_amd.engine import TF1_GRAD_F32, TF1_STATE_F32, TF1_W_F32
    rng = np.random.default_rng(1300)
    shapes = [(16, 1, 8), (8,), (168, 8), (8,)]
    n, rho, lr1, lr2 = 3, 0.99, 0.025, 0.001
    dt = {"32": np.float32, "64": np.float64}
    sd, gd, wd = dt[dtypes[1:3]], dt[dtypes[5:7]], dt[dtypes[9:11]]
    state_dtype = sd
    W4 = [rng.standard_normal(s).astype(wd) for s in shapes]
    st4 = [rng.standard_normal(s + (n,)).astype(sd) for s in shapes]
    g = [[rng.standard_normal(s).astype(gd) for s in shapes] for _ in range(n)]
    mask = (TF1_STATE_F32 if sd == np.float32 else 0) | (TF1_GRAD_F32 if gd == np.float32 else 0) | \
        (TF1_W_F32 if wd == np.float32 else 0)
    ref_states = [x.copy() for x in st4]
    ref_W = O.tf1_mewma([w.copy() for w in W4], ref_states, g, rho, lr1, lr2, filtered, init)
    from federated_amd.engine import BucketLayout
    lay = BucketLayout([s for s in shapes])
    dW = _dev64(lay.pack(W4, np.empty(lay.P)))
    ds = [_dev64(lay.pack([x[..., j] for x in st4], np.empty(lay.P))) for j in range(n)]
    dg = [_dev64(lay.pack(gj, np.empty(lay.P))) for gj in g]
    gpu.mewma_tf1_f64(dW, ds, dg, rho, lr1, lr2, int(lay.offsets[2]), init, filtered, mask)
    for k, (a, r) in enumerate(zip(lay.unpack(dW.cpu().numpy()), ref_W)):
        assert np.array_equal(a.astype(r.dtype), r) and np.array_equal(a, r.astype(np.float64)), (k, r.dtype)
    for j in range(n):
        for k, a in enumerate(lay.unpack(ds[j].cpu().numpy())):
            assert np.array_equal(a.astype(state_dtype), ref_states[k][..., j]), (j, k)
            assert np.array_equal(a, ref_states[k][..., j].astype(np.float64)), (j, k)


@pytest.mark.parametrize("rule", [0, 2, 3])
@pytest.mark.parametrize("n", [0, 1, 4, 17])
def test_fold_f64_rules(gpu, rule, n):
    """cfa_fold_f64: SEQUENTIAL / SEQUENTIAL_DIV / ACCUMULATE on fp64 buckets, identical to the
    numpy fp64 chain (one rounding per operation)."""
    rng = np.random.default_rng(1400 + 10 * rule + n)
    P = 20_003
    local = rng.standard_normal(P)
    xs = [rng.standard_normal(P) for _ in range(n)]
    a = [float(v) for v in rng.random(n)]
    d = [float(v) for v in rng.integers(1, 9, n)]
    ref = local.copy()
    for j in range(n):
        if rule == 0:
            ref = ref + a[j] * (xs[j] - ref)
        elif rule == 2:
            ref = ref + a[j] * (xs[j] - ref) / d[j]
        else:
            ref = ref + a[j] * xs[j]
    out = torch.empty(P, dtype=torch.float64, device="cuda")
    gpu.fold_f64(out, _dev64(local), [_dev64(x) for x in xs], a, rule, d if rule == 2 else None)
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("rule", [0, 2])
def test_fold_f64_grid_stride_large(gpu, rule):
    """A bucket of more full tiles than the grid has workgroups (each workgroup walks several, the
    partial tile and the odd last element apart), with the compression epilogue on a range that
    starts and ends inside tiles: identical to numpy (round 4 kernel skeleton, sc1 buffer store)."""
    rng = np.random.default_rng(1450 + rule)
    P, n = 4_000_003, 4
    local = rng.standard_normal(P) * 1e-3
    xs = [local + rng.standard_normal(P) * 1e-4 for _ in range(n)]
    a = [0.2, 0.3, 0.25, 0.1]
    d = [4.0, 3.0, 4.0, 7.0]
    ref = local.copy()
    for j in range(n):
        ref = ref + a[j] * (xs[j] - ref) / d[j] if rule == 2 else ref + a[j] * (xs[j] - ref)
    out = torch.empty(P, dtype=torch.float64, device="cuda")
    gpu.fold_f64(out, _dev64(local), [_dev64(x) for x in xs], a, rule, d if rule == 2 else None)
    assert np.array_equal(out.cpu().numpy(), ref)
    if rule == 0:  # the TF1 entry (same kernel) with the epilogue on [cb, ce)
        cb, ce = 1_000_001, 3_000_007
        y = O.tf1_mix_flat(local, xs, a)
        seg = y[cb:ce].reshape(1, -1)
        cnt = O.tf1_compress(seg, local[cb:ce].reshape(1, -1), 3)
        y[cb:ce] = seg.reshape(-1)
        kept = torch.zeros(1, dtype=torch.int64, device="cuda")
        gpu.mix_tf1_f64(out, _dev64(local), [_dev64(x) for x in xs], a, False, 3, cb, ce, kept)
        assert np.array_equal(out.cpu().numpy(), y) and int(kept.item()) == cnt


def test_mix_tf1_error_paths(gpu):
    from federated_amd._lib import CFAError
    x = torch.zeros(16, device="cuda")
    with pytest.raises(CFAError):
        gpu.mix_tf1(x, x, [x], [0.5])  # out aliases a neighbour
    with pytest.raises(CFAError):
        gpu.mix_tf1(x, torch.zeros(16, device="cuda"), [torch.zeros(16, device="cuda")], [0.5], 2, 0, 8)  # no kept
    with pytest.raises(CFAError):
        gpu.mix_tf1(x, torch.zeros(16, device="cuda"), [], [], 9, 0, 8, torch.zeros(1, dtype=torch.int64, device="cuda"))


@pytest.mark.parametrize("filtered,init", [(True, False), (False, False), (False, True)])
@pytest.mark.parametrize("n", [1, 2, 5])
def test_mewma_bitexact_fp32(gpu, filtered, init, n):
    rng = np.random.default_rng(400 + n)
    P, split = 1488 * 37 + 3, 136 * 37
    rho, lr1, lr2 = 0.99, 0.1, 0.05
    W = _rand(rng, 1, P)[0]
    s = _rand(rng, n, P)
    g = _rand(rng, n, P)
    # fp32 oracle: same op order as cfa_ge_2stage.py:594-621 on fp32 arrays
    Wr, sr = W.copy(), [x.copy() for x in s]
    lr = np.where(np.arange(P) < split, np.float32(lr1), np.float32(lr2)).astype(np.float32)
    for j in range(n):
        sr[j] = g[j].copy() if init else rho * g[j] + (1 - rho) * sr[j]
        Wr = Wr - lr * (sr[j] if filtered else g[j])
    dW, ds = _dev(W), [_dev(x) for x in s]
    gpu.mewma(dW, ds, [_dev(x) for x in g], rho, lr1, lr2, split, init, filtered)
    assert np.array_equal(dW.cpu().numpy(), Wr)
    for j in range(n):
        assert np.array_equal(ds[j].cpu().numpy(), sr[j])


def test_population_kernel_matches_per_device(gpu):
    """One launch over a k-regular population == per-device sequential mixes."""
    rng = np.random.default_rng(9)
    D, P, N = 12, 100_001, 4
    buckets = _rand(rng, D, P)
    dev = [_dev(b) for b in buckets]
    outs = [torch.empty(P, dtype=torch.float32, device="cuda") for _ in range(D)]
    ptr, idx, coef = [0], [], []
    expect = []
    for d in range(D):
        nbr = O.tf1_kregular(d, N, D).tolist()
        a = 1.0 / (len(nbr) + 1)
        idx += [d] + nbr
        coef += [1.0] + [a] * len(nbr)
        ptr.append(len(idx))
        expect.append(O.sequential_mix(buckets[d], [buckets[j] for j in nbr], [a] * len(nbr)))
    t64 = lambda xs: torch.tensor([x.data_ptr() for x in xs], dtype=torch.int64, device="cuda")
    gpu.population(t64(outs), t64(dev), torch.tensor(ptr, dtype=torch.int32, device="cuda"),
                   torch.tensor(idx, dtype=torch.int32, device="cuda"),
                   torch.tensor(coef, dtype=torch.float32, device="cuda"), D, 0, P)
    for d in range(D):
        assert np.array_equal(outs[d].cpu().numpy(), expect[d]), d


def test_full_size_properties(gpu):
    """BASELINE size (8 neighbours x 25M fp32): exact against the oracle over the whole bucket,
    plus size-independent properties (identity at a=0, convexity bound)."""
    P, n = 25_000_000, 8
    g = torch.Generator(device="cuda").manual_seed(20261015)
    local = torch.randn(P, generator=g, device="cuda")
    nbrs = [torch.randn(P, generator=g, device="cuda") for _ in range(n)]
    out = torch.empty_like(local)
    a = 1.0 / (n + 1)
    gpu.mix_seq(out, local, nbrs, [a] * n)
    lo = torch.minimum(local, torch.stack(nbrs).min(0).values)
    hi = torch.maximum(local, torch.stack(nbrs).max(0).values)
    assert bool(((out >= lo - 1e-6) & (out <= hi + 1e-6)).all())
    # the whole 25M bucket against the oracle, bit for bit (about a second of numpy)
    ref = O.sequential_mix(local.cpu().numpy(), [x.cpu().numpy() for x in nbrs], [a] * n)
    assert np.array_equal(out.cpu().numpy(), ref)
    gpu.mix_seq(out, local, nbrs[:1], [0.0])
    assert torch.equal(out, local)


def test_error_paths(gpu):
    from federated_amd import _lib
    x = torch.zeros(16, device="cuda")
    with pytest.raises(_lib.CFAError, match="aliases neighbour"):
        gpu.mix_seq(x, torch.zeros(16, device="cuda"), [x], [0.5])
    with pytest.raises(ValueError):
        gpu.mix_seq(x, torch.zeros(8, device="cuda"), [], [])
    with pytest.raises(TypeError):
        gpu.mix_seq(x, torch.zeros(16, device="cuda", dtype=torch.float64), [], [])


def test_arguments_on_another_gpu_are_refused(gpu, monkeypatch):
    """An engine bound to one GPU refuses tensors and streams of another before any launch (on a
    one-GPU box: the engine is told it runs on cuda:1, the arguments stay on cuda:0)."""
    monkeypatch.setattr(gpu, "device", torch.device("cuda", 1))
    x, y = torch.zeros(16, device="cuda:0"), torch.zeros(16, device="cuda:0")
    for call in (lambda: gpu.mix_seq(x, y, [y], [0.5]),
                 lambda: gpu.prepare_mix_seq(x, y, [y], [0.5]),
                 lambda: gpu.mix_seq_div(x, y, [y], [1.0], [2.0]),
                 lambda: gpu.mewma(x, [y], [y], 0.99, 0.1, 0.1, 16, False, True),
                 lambda: gpu.compress(x, None, 1, torch.zeros(1, dtype=torch.int64, device="cuda:0"))):
        with pytest.raises(ValueError, match="this engine runs on cuda:1"):
            call()


@pytest.mark.parametrize("n", [1, 3, 7, 20])
def test_mix_seq_div_bitexact(gpu, n):
    """FedAvg form p <- p + u*(x - p)/C (parameter_server_v2.py:159-161), fp32 numpy rounding."""
    rng = np.random.default_rng(600 + n)
    P = 1_000_003
    p = _rand(rng, 1, P)[0]
    xs = _rand(rng, n, P)
    for u in (1, 0.99):
        ref = O.ps_fedavg([p], [[x] for x in xs], u)[0]
        out = torch.empty(P, dtype=torch.float32, device="cuda")
        gpu.mix_seq_div(out, _dev(p), [_dev(x) for x in xs], [u] * n, [float(n)] * n)
        assert np.array_equal(out.cpu().numpy(), ref), (n, u)


def test_mix_seq_bucket_larger_than_2gib(gpu):
    """Buckets beyond the 32-bit buffer-offset range of the streaming store are split into
    <= 2 GiB launches; check windows at the start, around the chunk seam and at the end."""
    P = (1 << 29) + 12_345  # 2.15 GB per fp32 bucket
    g = torch.Generator(device="cuda").manual_seed(5)
    local = torch.randn(P, generator=g, device="cuda")
    nb = torch.randn(P, generator=g, device="cuda")
    out = torch.empty_like(local)
    gpu.mix_seq(out, local, [nb], [0.5])
    seam = 4 * (1 << 27)
    for a in (0, seam - 4096, P - 8192):
        sl = slice(a, a + 8192)
        ref = O.sequential_mix(local[sl].cpu().numpy(), [nb[sl].cpu().numpy()], [0.5])
        assert np.array_equal(out[sl].cpu().numpy(), ref), a
    del local, nb, out
    torch.cuda.empty_cache()


def _special(rng, P, dtype=np.float32):
    """Random values salted with the IEEE specials numpy meets in real weights: NaN, +-inf,
    -0.0, subnormals, the largest finite values."""
    fi = np.finfo(dtype)
    a = rng.standard_normal(P).astype(dtype)
    specials = np.array([np.nan, np.inf, -np.inf, -0.0, 0.0, fi.smallest_subnormal, -fi.smallest_subnormal,
                         fi.smallest_normal * 0.5, fi.tiny, fi.max, -fi.max, 1e-40 if dtype == np.float32 else 1e-310],
                        dtype=dtype)
    idx = rng.choice(P, size=min(P, 3 * len(specials)), replace=False)
    a[idx] = np.resize(specials, idx.size)
    return a


def _same_bits_or_nan(got, ref):
    """Bitwise equal, except that any NaN matches any NaN (payloads are not specified)."""
    got, ref = np.asarray(got), np.asarray(ref)
    both_nan = np.isnan(got) & np.isnan(ref)
    gi = got.view(np.uint32 if got.dtype == np.float32 else np.uint64)
    ri = ref.view(np.uint32 if ref.dtype == np.float32 else np.uint64)
    return bool(np.all(both_nan | (gi == ri)))


@pytest.mark.parametrize("n", [1, 3, 8])
def test_special_values_follow_numpy(gpu, n):
    """NaN / inf / -0.0 / subnormal inputs: the fp32 sequential rule, the FedAvg divisor rule and
    the TF1 fp64 chain give numpy's results (no flush-to-zero, IEEE inf/NaN propagation)."""
    rng = np.random.default_rng(700 + n)
    P = 4096 + 5
    local = _special(rng, P)
    nbrs = [_special(rng, P) for _ in range(n)]
    alphas = [1.0 / (n + 1)] * n
    with np.errstate(all="ignore"):
        ref = O.sequential_mix(local, nbrs, alphas)
    out = torch.empty(P, dtype=torch.float32, device="cuda")
    gpu.mix_seq(out, _dev(local), [_dev(x) for x in nbrs], alphas)
    assert _same_bits_or_nan(out.cpu().numpy(), ref)
    # FedAvg form p + u * (x - p) / C
    with np.errstate(all="ignore"):
        w = local.copy()
        for x in nbrs:
            w = w + np.float32(1.0) * (x - w) / np.float32(n)
    out2 = torch.empty(P, dtype=torch.float32, device="cuda")
    gpu.mix_seq_div(out2, _dev(local), [_dev(x) for x in nbrs], [1.0] * n, [float(n)] * n)
    assert _same_bits_or_nan(out2.cpu().numpy(), w)
    # TF1 fp64 chain on fp64 buckets of fp64 specials
    l64 = _special(rng, P, np.float64)
    n64 = [_special(rng, P, np.float64) for _ in range(n)]
    a64 = [0.5 / (k + 1) for k in range(n)]
    with np.errstate(all="ignore"):
        r64 = O.tf1_mix_flat(l64, n64, a64)
    o64 = torch.empty(P, dtype=torch.float64, device="cuda")
    gpu.mix_tf1_f64(o64, _dev(l64), [_dev(x) for x in n64], a64, False)
    assert _same_bits_or_nan(o64.cpu().numpy(), r64)


_RAND_DIVISORS = [float(v) for v in np.random.default_rng(4244).integers(0, 0x7F7FFFFF, 24, dtype=np.uint32)
                  .view(np.float32)]


@pytest.mark.parametrize("divisors", [[float(c) for c in range(1, 65)],
                                      [3.0, 7.0, 1e-7, 3e7, 0.1, 1023.0, 2.0 ** 20, 2.0 ** -20],
                                      [float(c) for c in (97, 255, 4095, 65535, 1048575)],
                                      [1e-40, 1.4e-45, -3.0, -0.1, 3.4028235e38, 1e-38, 0.0, -0.0, np.inf],
                                      _RAND_DIVISORS])
def test_mix_seq_div_quotient_exact_over_exponent_range(gpu, divisors):
    """The fold's division (one fp64 multiply by RN_64(1/C), cfa_internal.h div_rd) equals numpy's
    fp32 a / C bit for bit: with local = 0 and u = 1 the one-step fold is 0 + x / C, for x spread
    over every binade from 2^-149 to 2^127 (zeros, subnormals, the old Markstein guard's edges,
    infinities and NaN included) and divisors over every binade (subnormal, negative, the largest
    finite, zero and infinity included, plus 24 random fp32 bit patterns)."""
    rng = np.random.default_rng(4242)
    P = 1 << 22
    mant = rng.integers(0, 1 << 23, P, dtype=np.uint32)
    expo = rng.integers(0, 255, P, dtype=np.uint32)  # every biased exponent but inf/nan
    sign = rng.integers(0, 2, P, dtype=np.uint32) << 31
    x = (sign | (expo << 23) | mant).view(np.float32)
    edges = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 2.0 ** -100, -(2.0 ** -100), 2.0 ** 100,
                      np.nextafter(np.float32(2.0 ** -100), np.float32(0)), np.nextafter(np.float32(2.0 ** 100),
                                                                                  np.float32(np.inf)),
                      1.0, 3.0, 1e-45, 3.4028235e38], dtype=np.float32)
    x[:edges.size] = edges
    xd = _dev(x)
    zero = torch.zeros(P, device="cuda")
    out = torch.empty(P, device="cuda")
    with np.errstate(all="ignore"):
        for C in divisors:
            gpu.mix_seq_div(out, zero, [xd], [1.0], [C])
            ref = np.float32(0.0) + (np.float32(1.0) * (x - np.float32(0.0))) / np.float32(C)
            got = out.cpu().numpy()
            same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
            assert same.all(), (C, x[~same][:4], got[~same][:4], ref[~same][:4])


@pytest.mark.parametrize("o", [49, 75, 77, 1, 3, 1023, 4095])
def test_mix_seq_div_exact_subnormal_ties(gpu, o):
    """Quotients exactly on a subnormal rounding midpoint (round-4 advisor finding): x = k * o *
    2^-149 for odd k, C = 2 o, so x / C = (k / 2) * 2^-149 and ties-to-even decides. The fold's
    one-multiply division alone rounds some of these the wrong way; div_rd sends 0 < |p| < 2^-126 to
    the IEEE division. Random bit patterns (the test above) practically never hit these."""
    k = np.arange(1, 1 << 15, 2, dtype=np.float64)
    k = k[k * o < 2 ** 24]
    x = np.concatenate([k * o * 2.0 ** -149, -(k * o * 2.0 ** -149)]).astype(np.float32)
    x = np.concatenate([x, np.zeros((-x.size) % 64 + 64, np.float32)])  # 64-aligned, a zero tail
    P = x.size
    zero = torch.zeros(P, device="cuda")
    out = torch.empty(P, device="cuda")
    gpu.mix_seq_div(out, zero, [_dev(x)], [1.0], [float(2 * o)])
    ref = np.float32(0.0) + (np.float32(1.0) * (x - np.float32(0.0))) / np.float32(2 * o)
    got = out.cpu().numpy()
    same = got.view(np.uint32) == ref.view(np.uint32)
    assert same.all(), (o, x[~same][:4], got[~same][:4], ref[~same][:4])


@pytest.mark.parametrize("divisors", [[float(c) for c in range(1, 33)], [3.0, 1e-6, 7e5, 0.1, 2.0 ** 20, 2.0 ** -20]])
def test_fold_f64_div_quotient_exact_over_exponent_range(gpu, divisors):
    """fp64 divisor fold (cfa_fold_f64, SEQUENTIAL_DIV): with local = 0 and u = 1 the one-step
    fold is 0 + x / C; equal to numpy's fp64 division bit for bit for x over every binade,
    zeros, subnormals, the guard's edges, infinities and NaN."""
    import torch
    from federated_amd import _lib
    rng = np.random.default_rng(4343)
    P = 1 << 21
    mant = rng.integers(0, 1 << 52, P, dtype=np.uint64)
    expo = rng.integers(0, 2047, P, dtype=np.uint64)
    sign = rng.integers(0, 2, P, dtype=np.uint64) << np.uint64(63)
    x = (sign | (expo << np.uint64(52)) | mant).view(np.float64)
    edges = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 2.0 ** -900, 2.0 ** 900, -(2.0 ** 900),
                      np.nextafter(2.0 ** -900, 0.0), np.nextafter(2.0 ** 900, np.inf), 5e-324, 1.7976931348623157e308,
                      1.0, 3.0])
    x[:edges.size] = edges
    xd = torch.from_numpy(x).cuda()
    zero = torch.zeros(P, dtype=torch.float64, device="cuda")
    out = torch.empty(P, dtype=torch.float64, device="cuda")
    with np.errstate(all="ignore"):
        for C in divisors:
            gpu.fold_f64(out, zero, [xd], [1.0], _lib.RULE_SEQUENTIAL_DIV, [C])
            ref = 0.0 + (1.0 * (x - 0.0)) / C
            got = out.cpu().numpy()
            same = (got.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(got) & np.isnan(ref))
            assert same.all(), (C, x[~same][:4], got[~same][:4], ref[~same][:4])


@pytest.mark.parametrize("n,P,off,mode", [(2, 16_680, 0, 0), (3, 24_622, 0, 2), (1, 1001, 1, 1), (19, 5003, 0, 3),
                                          (4, 4099, 3, 4)])
def test_tf1_wide_equals_f64_rows(gpu, n, P, off, mode):
    """cfa_mix_tf1_wide_f32 (fp32 rows in, unrounded fp64 out) equals cfa_mix_tf1_f64 on the same
    rows widened to fp64 with step0_f32 (the reference's numpy-2 chain for fp32 inputs), bit for
    bit, counts included: misaligned starts, fan-in above CFA_MAX_FANIN (chained in the output)
    and every compression mode."""
    from federated_amd import _lib
    g = torch.Generator(device="cuda").manual_seed(P + n)
    base = torch.randn((n + 1) * (P + 8), device="cuda", generator=g) * 1e-3
    rows = [base[j * (P + 8) + off: j * (P + 8) + off + P] for j in range(n + 1)]
    al = [0.5 / (n + 1)] * n
    cb, ce = (P // 3, min(P, P // 3 + 777)) if mode else (0, 0)
    out_w = torch.full((P + 1,), float("nan"), dtype=torch.float64, device="cuda")[1:] if off else \
        torch.full((P,), float("nan"), dtype=torch.float64, device="cuda")
    kw, kf = gpu.counter(), gpu.counter()
    _lib.call("cfa_mix_tf1_wide_f32", out_w.data_ptr(), rows[0].data_ptr(),
              _lib.ptr_table([r.data_ptr() for r in rows[1:]]), _lib.double_array(al), n, P, mode, cb, ce,
              kw.data_ptr() if mode else None, gpu.stream_handle())
    r64 = [r.double() for r in rows]
    out_f = torch.empty(P, dtype=torch.float64, device="cuda")
    gpu.mix_tf1_f64(out_f, r64[0], r64[1:], al, True, mode, cb, ce, kf if mode else None)
    torch.cuda.synchronize()
    assert torch.equal(out_w, out_f)
    assert int(kw.item()) == int(kf.item())


@pytest.mark.parametrize("where", ["local", "nbr_tail", "nbr_head", "local_start"])
def test_tf1_wide_rejects_fp64_out_overlapping_inputs(gpu, where):
    """The fp64 out is 8P bytes: any overlap with an fp32 input range is refused before launch
    (ADVICE r02), not only an out that starts at a neighbour."""
    from federated_amd import _lib
    P = 1024
    buf = torch.zeros(8 * P, device="cuda")  # room for every layout below
    local, nbr = buf[:P], buf[4 * P:5 * P]
    base = buf.data_ptr()
    out_ptr = {"local": base + 8,                       # inside local
               "nbr_tail": base + 4 * P * 4 - 8 * P + 16,  # its tail reaches the neighbour
               "nbr_head": base + 4 * P * 4 + 8,  # starts inside the neighbour
               "local_start": base}[where]
    with pytest.raises(_lib.CFAError, match="overlaps"):
        _lib.call("cfa_mix_tf1_wide_f32", out_ptr, local.data_ptr(), _lib.ptr_table([nbr.data_ptr()]),
                  _lib.double_array([0.5]), 1, P, 0, 0, 0, None, gpu.stream_handle())
    ok = torch.empty(P, dtype=torch.float64, device="cuda")
    _lib.call("cfa_mix_tf1_wide_f32", ok.data_ptr(), local.data_ptr(), _lib.ptr_table([nbr.data_ptr()]),
              _lib.double_array([0.5]), 1, P, 0, 0, 0, None, gpu.stream_handle())
    torch.cuda.synchronize()


def test_full_size_tf1_wide_and_sharded_fedavg(gpu):
    """BASELINE size (8 neighbours x 25M): the TF1 wide kernel against the oracle's fp64 chain
    over the whole bucket, bit for bit (fp32 arrays in, the reference's fp64 result out), and
    the sharded-FedAvg closed form (cfa_mix_f32 over 8 models + the global one) within 1e-5
    normwise of the sequential FedAvg fold."""
    from federated_amd import _lib
    from federated_amd.ps_shard import ShardedFedAvg
    P, n = 25_000_000, 8
    g = torch.Generator(device="cuda").manual_seed(20261016)
    rows = torch.randn(n + 1, P, generator=g, device="cuda")
    al = [0.5 / (n + 1)] * n
    out = torch.empty(P, dtype=torch.float64, device="cuda")
    _lib.call("cfa_mix_tf1_wide_f32", out.data_ptr(), rows[0].data_ptr(),
              _lib.ptr_table([rows[j].data_ptr() for j in range(1, n + 1)]), _lib.double_array(al), n, P, 0, 0, 0,
              None, gpu.stream_handle())
    h = rows.cpu().numpy()
    ref = O.tf1_mix_flat(h[0], [h[j] for j in range(1, n + 1)], al)
    torch.cuda.synchronize()
    assert ref.dtype == np.float64 and np.array_equal(out.cpu().numpy(), ref)
    del out
    ps = ShardedFedAvg(0, 1, n, P, "cuda", None, gpu, update_factor=1.0)
    ps.models.copy_(rows[1:])
    ps.params.copy_(rows[0])
    got = ps.aggregate().cpu().numpy()
    ref = O.ps_fedavg([h[0]], [[h[j]] for j in range(1, n + 1)], 1.0)[0]
    assert np.max(np.abs(got - ref)) <= 1e-5 * np.max(np.abs(ref))
