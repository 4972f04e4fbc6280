"""(f3) HIP gradient kernels (cfa_ge_grad_cnn_f32 / cfa_ge_grad_2nn_f32) against the oracle's
float64 gradients of the TF1 graphs (cfa_ge_2stage.py:391-433): fp32 kernels, tolerance
1e-5 normwise per tensor (max|g - r| <= 1e-5 max|r|, the north-star fp32 bar)."""
import numpy as np
import pytest

from conftest import normwise_close
from oracle import cfa_oracle as orc

pytestmark = pytest.mark.gpu


def _cnn_models(rng, M, F=16, NC=8, LN=168, C=8):
    return [[(rng.standard_normal((F, 1, NC)) * 0.3).astype(np.float32),
             (rng.standard_normal(NC) * 0.1).astype(np.float32),
             (rng.standard_normal((LN, C)) * 0.1).astype(np.float32),
             (rng.standard_normal(C) * 0.1).astype(np.float32)] for _ in range(M)]


def _check(got, models, ref_fn):
    for g, m in zip(got, models):
        ref, _ = ref_fn(m)
        for a, r in zip(g, ref):
            assert a.dtype == np.float32 and a.shape == r.shape
            assert normwise_close(a, r, 1e-5), (np.abs(a - r).max(), np.abs(r).max())


@pytest.mark.parametrize("B,M", [(24, 2), (24, 5), (1, 1), (100, 3)])  # 100: chunked through LDS
def test_cnn_gradients_match_oracle(gpu, B, M):
    from federated_amd.consensus import _tf1_models as T
    rng = np.random.default_rng(B * 10 + M)
    models = _cnn_models(rng, M)
    x = rng.standard_normal((B, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[rng.integers(0, 8, B)]
    got = T.gradients_batched(1, x, y, models, stride=5)
    _check(got, models, lambda m: orc.tf1_cnn_grads(x, y, *m, stride=5))


@pytest.mark.parametrize("L,S,F", [(100, 3, 5), (64, 2, 7), (37, 4, 4)])
def test_cnn_other_geometries(gpu, L, S, F):
    from federated_amd.consensus import _tf1_models as T
    rng = np.random.default_rng(L)
    L2 = -(-(-(-L // S)) // S)
    models = _cnn_models(rng, 2, F=F, NC=6, LN=L2 * 6, C=5)
    x = rng.standard_normal((9, L)).astype(np.float32)
    y = np.eye(5, dtype=np.float32)[rng.integers(0, 5, 9)]
    got = T.gradients_batched(1, x, y, models, stride=S)
    _check(got, models, lambda m: orc.tf1_cnn_grads(x, y, *m, stride=S))


@pytest.mark.parametrize("B,M", [(24, 2), (300, 2), (3, 4)])  # 300: chunked through LDS
def test_2nn_gradients_match_oracle(gpu, B, M):
    from federated_amd.consensus import _tf1_models as T
    rng = np.random.default_rng(B + M)
    models = [[(rng.standard_normal((512, 32)) * 0.1).astype(np.float32),
               (rng.standard_normal(32) * 0.1).astype(np.float32),
               (rng.standard_normal((32, 8)) * 0.3).astype(np.float32),
               (rng.standard_normal(8) * 0.1).astype(np.float32)] for _ in range(M)]
    x = rng.standard_normal((B, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[rng.integers(0, 8, B)]
    got = T.gradients_batched(2, x, y, models)
    _check(got, models, lambda m: orc.tf1_2nn_grads(x, y, *m))


def test_saturated_softmax(gpu):
    from federated_amd.consensus import _tf1_models as T
    rng = np.random.default_rng(9)
    models = _cnn_models(rng, 1)
    models[0][3] = np.array([40, 0, 0, 0, 0, 0, 0, 0], np.float32)
    x = rng.standard_normal((6, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[[0, 0, 1, 0, 2, 0]]
    got = T.gradients_batched(1, x, y, models, stride=5)
    _check(got, models, lambda m: orc.tf1_cnn_grads(x, y, *m, stride=5))


def test_bad_geometry_is_refused(gpu):
    from federated_amd.consensus import _tf1_models as T
    rng = np.random.default_rng(1)
    models = _cnn_models(rng, 1, LN=160)  # multip 20 != ceil(ceil(512/5)/5) = 21
    x = rng.standard_normal((2, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[[0, 1]]
    with pytest.raises(ValueError):
        T.gradients_batched(1, x, y, models, stride=5)


@pytest.mark.parametrize("ml,B,M", [(1, 24, 3), (2, 24, 3), (1, 5, 40), (2, 100, 2)])
def test_rows_form_with_and_without_batch_split(gpu, ml, B, M):
    """cfa_ge_grad_*_rows_f32: evaluation m = data row drow[m] at model row mrow[m]; with a
    workspace the batch is split over workgroups and summed in a second pass."""
    import torch
    rng = np.random.default_rng(ml * 100 + B + M)
    Dx, Dm = 3, 4
    if ml == 1:
        geom = {"filter": 16, "number": 8, "stride": 5}
        models = _cnn_models(rng, Dm)
        ref_fn = lambda xi, yi, m: orc.tf1_cnn_grads(xi, yi, *m, stride=5)
    else:
        geom = {"intermediate_nodes": 32}
        models = [[(rng.standard_normal((512, 32)) * 0.1).astype(np.float32), (rng.standard_normal(32) * 0.1).astype(np.float32),
                   (rng.standard_normal((32, 8)) * 0.3).astype(np.float32), (rng.standard_normal(8) * 0.1).astype(np.float32)]
                  for _ in range(Dm)]
        ref_fn = lambda xi, yi, m: orc.tf1_2nn_grads(xi, yi, *m)
    flat = np.stack([np.concatenate([a.reshape(-1) for a in m]) for m in models])
    P = flat.shape[1]
    x = rng.standard_normal((Dx, B, 512)).astype(np.float32)
    y = np.eye(8, dtype=np.float32)[rng.integers(0, 8, (Dx, B))]
    mrow = rng.integers(0, Dm, M).astype(np.int32)
    drow = rng.integers(0, Dx, M).astype(np.int32)
    t = lambda a: torch.from_numpy(a).cuda()
    outs = []
    for ws in (None, gpu.grad_workspace(M, B, P)):
        g = torch.empty(M, P, device="cuda")
        gpu.grad_rows(ml, t(x), t(y), t(flat), t(mrow), t(drow), g, geom, workspace=ws)
        outs.append(g.cpu().numpy())
    offs = np.concatenate([[0], np.cumsum([a.size for a in models[0]])])
    for out in outs:
        for m in range(M):
            ref, _ = ref_fn(x[drow[m]], y[drow[m]], models[mrow[m]])
            for k in range(4):
                assert normwise_close(out[m, offs[k]:offs[k + 1]], ref[k].reshape(-1), 1e-5), (m, k)


@pytest.mark.parametrize("ml", [1, 2])
def test_split_launch_reuses_its_workspace(gpu, ml):
    """Back-to-back split launches on one workspace give the same bits every time, and agree with
    the unsplit launch within the tolerance."""
    import torch
    rng = np.random.default_rng(50 + ml)
    D, B, M = 16, 24, 32
    if ml == 1:
        geom, P = {"filter": 16, "number": 8, "stride": 5}, 16 * 8 + 8 + 21 * 8 * 8 + 8
    else:
        geom, P = {"intermediate_nodes": 32}, 512 * 32 + 32 + 32 * 8 + 8
    x = torch.from_numpy(rng.standard_normal((D, B, 512)).astype(np.float32)).cuda()
    y = torch.from_numpy(np.eye(8, dtype=np.float32)[rng.integers(0, 8, (D, B))]).cuda()
    models = torch.from_numpy((rng.standard_normal((D, P)) * 0.1).astype(np.float32)).cuda()
    mrow = torch.from_numpy(rng.integers(0, D, M).astype(np.int32)).cuda()
    drow = torch.from_numpy(np.repeat(np.arange(D), 2).astype(np.int32)).cuda()
    ws = gpu.grad_workspace(M, B, P)
    assert ws.numel() >= 2 * M * P  # config 3 shapes do split
    outs = []
    for _ in range(4):
        g = torch.full((M, P), float("nan"), device="cuda")
        gpu.grad_rows(ml, x, y, models, mrow, drow, g, geom, workspace=ws)
        outs.append(g)
    torch.cuda.synchronize()
    for g in outs[1:]:
        assert torch.equal(g, outs[0])
    single = torch.empty(M, P, device="cuda")
    gpu.grad_rows(ml, x, y, models, mrow, drow, single, geom)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    assert float((outs[0] - single).abs().max()) <= 1e-5 * float(single.abs().max())
