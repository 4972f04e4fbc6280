"""GPU tests of the population round, the RCCL transport owned by libcfa (world_size 1: grouped
self send/recv + all-reduce through the C-ABI) and the host-staging path."""
import numpy as np
import pytest
import torch

from oracle.cfa_oracle import sequential_mix

pytestmark = pytest.mark.gpu


def test_ring_population_round_world1(gpu):
    from federated_amd.population import RingPopulationShard, RingShardPlan
    plan = RingShardPlan(0, 1, 12, 4)
    shard = RingPopulationShard(plan, 50_003, torch.device("cuda"), None, gpu)
    shard.models.normal_()
    shard.round()
    torch.cuda.synchronize()
    host = shard.models.cpu().numpy()
    mixed = shard.mixed.cpu().numpy()
    for i in range(plan.L):
        ref = sequential_mix(host[i], [host[j] for j in plan.neighbours(i)], shard.alphas)
        assert np.array_equal(mixed[i], ref), i


def test_rccl_transport_world1():
    from federated_amd.dist import RcclTransport
    t = RcclTransport(0, 1, 0)
    try:
        a = torch.randn(100_003, device="cuda")
        b = torch.empty_like(a)
        c = torch.randn(7, device="cuda")
        d = torch.empty_like(c)
        t.exchange([(a, 0)], [(b, 0)])
        torch.cuda.synchronize()
        assert torch.equal(a, b)
        with pytest.raises(ValueError):
            t.exchange([(a, 0)], [(d, 0)])
        ref = c.clone()
        t.allreduce_sum(c)
        torch.cuda.synchronize()
        assert torch.equal(c, ref)
    finally:
        t.close()


def test_rccl_p2p_group_world1_ragged_messages():
    """cfa_p2p_group_f32 (the routed halo's step): several self messages of different lengths
    and 256-byte-aligned offsets into one buffer, paired in issue order; a prepared group runs
    twice with the same tables; zero-length messages are skipped."""
    from federated_amd.dist import RcclTransport
    t = RcclTransport(0, 1, 0)
    try:
        src = torch.randn(3 * 4096 + 123, device="cuda")
        dst = torch.zeros_like(src)
        cuts = [0, 4096, 4096, 2 * 4096 + 64, src.numel()]
        sends = [(src[a:b], 0) for a, b in zip(cuts, cuts[1:])]
        recvs = [(dst[a:b], 0) for a, b in zip(cuts, cuts[1:])]
        run = t.prepare(sends, recvs)
        run()
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
        src.normal_()
        run(torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
        with pytest.raises(ValueError):
            t.prepare(sends, recvs[::-1])
    finally:
        t.close()


def test_population_shard_with_rccl_transport_world1(gpu):
    """world_size 1 never exchanges; the transport object is accepted and idle."""
    from federated_amd.dist import RcclTransport
    from federated_amd.population import RingPopulationShard, RingShardPlan
    t = RcclTransport(0, 1, 0)
    try:
        plan = RingShardPlan(0, 1, 10, 2)
        shard = RingPopulationShard(plan, 4096, torch.device("cuda"), t, gpu)
        shard.models.normal_()
        shard.round()
        torch.cuda.synchronize()
        h = shard.models.cpu().numpy()
        assert np.array_equal(shard.mixed[3].cpu().numpy(),
                              sequential_mix(h[3], [h[j] for j in plan.neighbours(3)], shard.alphas))
    finally:
        t.close()


def test_host_staging_e2e_small(gpu):
    from federated_amd.staging import measure_e2e
    r = measure_e2e(gpu, 1_000_003, 4, reps=2, chunks=4)
    assert r["pipelined_equals_device_result"]
    assert r["zero_copy_equals_device_result"]
    assert r["serial"]["ms"] > 0 and r["h2d_GBps"] > 0 and r["zero_copy"]["ms"] > 0


@pytest.mark.parametrize("P,n", [(1, 1), (4099, 3), (262_147, 8)])
def test_mix_seq_pinned_host_buckets(gpu, P, n):
    """Zero-copy form (f2): the kernel reads pinned host buckets over PCIe and writes the pinned
    host output; bit-exact against the oracle's sequential rule."""
    g = torch.Generator().manual_seed(P + n)
    local = torch.randn(P, generator=g).pin_memory()
    nbrs = [torch.randn(P, generator=g).pin_memory() for _ in range(n)]
    out = torch.full((P,), float("nan")).pin_memory()
    alphas = [1.0 / (n + 1)] * n
    gpu.mix_seq_pinned(out, local, nbrs, alphas)
    torch.cuda.synchronize()
    ref = sequential_mix(local.numpy(), [x.numpy() for x in nbrs], alphas)
    assert np.array_equal(out.numpy(), ref)


def test_mix_seq_pinned_rejects_pageable_and_device_tensors(gpu):
    with pytest.raises(ValueError):
        gpu.mix_seq_pinned(torch.empty(8).pin_memory(), torch.empty(8), [torch.empty(8).pin_memory()], [0.5])
    with pytest.raises(ValueError):
        gpu.mix_seq_pinned(torch.empty(8).pin_memory(), torch.empty(8, device="cuda"),
                           [torch.empty(8).pin_memory()], [0.5])


def _pop_tables(L, plan_or_lists, alphas_fn, buckets, outs):
    ptr, idx, coef = [0], [], []
    for i in range(L):
        nbr = plan_or_lists(i)
        idx += [i] + list(nbr)
        coef += [1.0] + alphas_fn(len(nbr))
        ptr.append(len(idx))
    t64 = lambda xs: torch.tensor([x.data_ptr() for x in xs], dtype=torch.int64, device="cuda")
    return (t64(outs), t64(buckets), torch.tensor(ptr, dtype=torch.int32, device="cuda"),
            torch.tensor(idx, dtype=torch.int32, device="cuda"),
            torch.tensor(coef, dtype=torch.float32, device="cuda"))


@pytest.mark.parametrize("name,D,P,nbr_fn,alpha_fn", [
    # config 2: FL_CFA_CNN_tf2 shapes (P = 24 622), 8 devices, K = 3 (cfa_ongraphs alpha = eps/(1+n))
    ("cfg2_cnn_8dev_K3", 8, 24_622, lambda i, D: [(i + o) % D for o in (-1, 1, 2)], lambda n: [1.0 / (1 + n)] * n),
    # config 3 topology: CFA-GE CNN (P = 1 488), 16 devices, k-regular N = 2 (cfa.py alpha 1/N)
    ("cfg3_cnn_ge_16dev", 16, 1_488, None, lambda n: [0.5] * n),
    # config 4: CIFAR-100 VGG-1 (P = 1 071 748), 32 devices, K = 4 ring window, eps = 1/(K+1)
    ("cfg4_vgg1_32dev_K4", 32, 1_071_748, lambda i, D: [(i + o) % D for o in (-2, -1, 1, 2)], lambda n: [1.0 / (n + 1)] * n),
    # config 5: radar (P = 24 622), 128 devices, ring in-neighbour ii-1 (consensus_v4 N < 2), eps = 1/2
    ("cfg5_radar_128dev_ring", 128, 24_622, lambda i, D: [(i - 1) % D], lambda n: [1.0 / (n + 1)] * n),
])
def test_config_shapes_population_kernel(gpu, name, D, P, nbr_fn, alpha_fn):
    """The functional BASELINE configs as one-launch population rounds (cfa_mix_population_f32),
    bit-exact against per-device sequential mixes on the oracle."""
    from oracle.cfa_oracle import tf1_kregular
    if nbr_fn is None:
        nbr_fn = lambda i, D: tf1_kregular(i, 2, D).tolist()
    g = torch.Generator(device="cuda").manual_seed(D * 7 + P)
    buckets = [torch.randn(P, generator=g, device="cuda") for _ in range(D)]
    outs = [torch.empty(P, device="cuda") for _ in range(D)]
    tables = _pop_tables(D, lambda i: nbr_fn(i, D), alpha_fn, buckets, outs)
    gpu.population(*tables, D, 0, P)
    torch.cuda.synchronize()
    host = [b.cpu().numpy() for b in buckets]
    for i in range(D):
        nbr = nbr_fn(i, D)
        ref = sequential_mix(host[i], [host[j] for j in nbr], alpha_fn(len(nbr)))
        assert np.array_equal(outs[i].cpu().numpy(), ref), (name, i)


@pytest.mark.parametrize("P", [1, 3, 4, 6, 1029, 2 * 256 * 4 + 3])
def test_population_kernel_small_and_ragged(gpu, P):
    """Buckets with no float4 body (P < 4) and ragged tails: the scalar tail runs inside the
    population launch (first tile column) and must round like the float4 body."""
    D = 5
    g = torch.Generator(device="cuda").manual_seed(P)
    buckets = [torch.randn(P, generator=g, device="cuda") for _ in range(D)]
    outs = [torch.empty(P, device="cuda") for _ in range(D)]
    nbr_fn = lambda i: [(i + o) % D for o in (-1, 1, 2)]
    alpha_fn = lambda n: [1.0 / (n + 1)] * n
    tables = _pop_tables(D, nbr_fn, alpha_fn, buckets, outs)
    gpu.population(*tables, D, 0, P)
    torch.cuda.synchronize()
    host = [b.cpu().numpy() for b in buckets]
    for i in range(D):
        ref = sequential_mix(host[i], [host[j] for j in nbr_fn(i)], alpha_fn(3))
        assert np.array_equal(outs[i].cpu().numpy(), ref), (P, i)


def test_config5_ring_round_world1(gpu):
    """Config 5 topology through the shard round (one-sided ring window)."""
    from federated_amd.population import RingPopulationShard, RingShardPlan
    plan = RingShardPlan(0, 1, 128, 1, 0)
    shard = RingPopulationShard(plan, 24_622, torch.device("cuda"), None, gpu)
    shard.models.normal_()
    shard.round()
    torch.cuda.synchronize()
    h = shard.models.cpu().numpy()
    out = shard.mixed.cpu().numpy()
    assert shard.alphas == [0.5]
    for i in (0, 1, 77, 127):
        assert np.array_equal(out[i], sequential_mix(h[i], [h[(i - 1) % 128]], [0.5]))


@pytest.mark.parametrize("P,placed", [(24_622, 0), (2_100_003, 0), (2_100_003, 2)])  # one population launch /
def test_graph_population_round_world1(gpu, P, placed):                         # per-device streaming mixes
    """Arbitrary topology (vGraph rows with the random.choices draw) as one shard: the round
    equals per-device sequential mixes on the oracle, bit for bit."""
    import random as _random
    from federated_amd import topology as T
    from federated_amd.graph_population import GraphPopulationShard, GraphShardPlan
    rng = np.random.default_rng(9)
    D = 12
    g = (rng.random((D, D)) < 0.4).astype(np.uint8)
    g = np.maximum(g, g.T)
    np.fill_diagonal(g, 0)
    lists = T.mobile(g[:, :, None], 0, 3, rng=_random.Random(3))
    plan = GraphShardPlan(lists, 0, 1)
    shard = GraphPopulationShard(plan, P, torch.device("cuda"), None, gpu, placement_candidates=placed)
    assert (shard.placement is not None) == bool(placed)
    shard.models.normal_()
    shard.round()
    torch.cuda.synchronize()
    h = shard.models.cpu().numpy()
    out = shard.mixed.cpu().numpy()
    for i in range(D):
        nb = lists[i]
        assert np.array_equal(out[i], sequential_mix(h[i], [h[j] for j in nb], T.alphas_tf2(nb, i, D))), i


@pytest.mark.parametrize("L,hl,hr,B,P", [(16, 4, 4, 8, 100_000), (13, 4, 4, 8, 24_622), (12, 2, 2, 8, 1_071_748 // 16),
                                         (10, 1, 0, 8, 24_622), (9, 3, 1, 4, 4097), (7, 0, 2, 1, 1003)])
def test_window_batched_round_equals_per_device(gpu, L, hl, hr, B, P):
    """cfa_mix_window_f32 passes (each window row loaded once for B devices) give the per-device
    mixes bit for bit: aligned rows (vector body), misaligned row pitches (scalar path), tails."""
    from federated_amd.population import RingPopulationShard, RingShardPlan
    plan = RingShardPlan(0, 1, L, hl, hr)
    a = RingPopulationShard(plan, P, torch.device("cuda"), None, gpu)
    b = RingPopulationShard(plan, P, torch.device("cuda"), None, gpu, window_batch=B)
    a.models.normal_()
    b.models.copy_(a.models)
    a.round()
    b.round()
    torch.cuda.synchronize()
    assert torch.equal(a.mixed, b.mixed)
    h = a.models.cpu().numpy()
    i = L // 2
    assert np.array_equal(b.mixed[i].cpu().numpy(), sequential_mix(h[i], [h[j] for j in plan.neighbours(i)], a.alphas))


def test_window_error_paths(gpu):
    from federated_amd._lib import CFAError
    x = [torch.zeros(64, device="cuda") for _ in range(20)]
    with pytest.raises(CFAError):  # nb > 8
        gpu.mix_window(x[:9], x[9:20], [[0.5, 0.5]] * 9, 1, 1)
    with pytest.raises(CFAError):  # output aliases a row
        gpu.mix_window([x[1]], x[0:3], [[0.5, 0.5]], 1, 1)
    with pytest.raises(ValueError):  # per-step alphas differ
        gpu.mix_window([x[10]], x[0:3], [[0.5, 0.25]], 1, 1)


@pytest.mark.parametrize("D,P,hl,hr", [(32, 1_071_748 // 8, 2, 2), (128, 24_622, 1, 0), (19, 50_001, 4, 4),
                                      (32, 1_071_748, 2, 2)])
def test_population_round_window_path_equals_csr(gpu, D, P, hl, hr):
    """topology.PopulationRound on a ring window runs the window passes (one
    cfa_mix_ring_round_f32 launch for 16-byte rows, cfa_mix_window_f32 passes otherwise);
    identical to the CSR one-launch kernel and to the oracle."""
    from federated_amd import topology as T
    lists = [[(d + o) % D for o in list(range(-hl, 0)) + list(range(1, hr + 1))] for d in range(D)]
    models = torch.randn(D, P, device="cuda")
    win = T.PopulationRound(gpu, models)
    win.set_topology(lists, T.alphas_tf2, use_window=True)
    assert win.window is not None and win.window[:2] == (hl, hr)
    auto = T.PopulationRound(gpu, models)
    auto.set_topology(lists, T.alphas_tf2)
    assert (auto.window is not None) == (P > T.WINDOW_MIN_P)
    csr = T.PopulationRound(gpu, models)
    csr.set_topology(lists, T.alphas_tf2, use_window=False)
    win.run()
    csr.run()
    torch.cuda.synchronize()
    assert torch.equal(win.out, csr.out)
    h = models.cpu().numpy()
    for d in (0, D // 2, D - 1):
        assert np.array_equal(win.out[d].cpu().numpy(), sequential_mix(h[d], [h[j] for j in lists[d]], T.alphas_tf2(lists[d], d, D)))


@pytest.mark.parametrize("divide", [False, True])
@pytest.mark.parametrize("zero_copy", [True, False])
def test_hostmixer_pipeline_equals_single_shot(gpu, monkeypatch, divide, zero_copy):
    """HostMixer.mix's chunked pipeline (chunk-major staging; each chunk mixed in place in pinned
    host memory, or moved by one H2D per chunk over three streams) returns the single-shot
    result bit for bit, across layer boundaries and ragged tails."""
    from federated_amd.consensus import _runtime as R
    monkeypatch.setattr(R, "PIPELINE_ZERO_COPY", zero_copy)
    monkeypatch.setattr(R, "NATIVE_PIPELINE", False)
    rng = np.random.default_rng(21)
    shapes = [(1001, 333), (333,), (517, 129), (7,)]
    local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(3)]
    al = [0.25, 0.5, 0.125]
    div = [4.0, 4.0, 4.0] if divide else None
    mx = R.mixer()
    ref, _ = mx.mix(local, nbrs, al, divisors=div)  # single shot (below the default threshold)
    monkeypatch.setattr(R, "PIPELINE_MIN_BYTES", 1 << 20)
    monkeypatch.setattr(R, "PIPELINE_CHUNK_BYTES", 600_000)
    got, kept = mx.mix(local, nbrs, al, divisors=div)
    assert kept is None
    for a, r, s in zip(got, ref, shapes):
        assert a.shape == s and a.dtype == np.float32 and np.array_equal(a, r)
    flat = lambda m: np.concatenate([x.reshape(-1) for x in m])
    if not divide:
        assert np.array_equal(flat(got), sequential_mix(flat(local), [flat(m) for m in nbrs], al))


@pytest.mark.parametrize("divide", [False, True])
@pytest.mark.parametrize("chunk,threads", [(4, 1), (1000, 3), (65_536, 8), (1 << 22, 16)])
def test_hostmixer_native_pipeline_equals_single_shot(gpu, monkeypatch, divide, chunk, threads):
    """cfa_host_mix_f32 (pack by host threads / zero-copy kernel / unpack, chunk by chunk, one
    call) returns the single-shot result bit for bit: chunks from 4 elements (every layer boundary
    inside a chunk, thousands of chunks) to one chunk, 1 to 16 copy threads, the FedAvg divisor
    form, fp64 and non-contiguous inputs, an empty layer."""
    from federated_amd.consensus import _runtime as R
    rng = np.random.default_rng(22)
    shapes = [(1001, 333), (0,), (333,), (517, 129), (7,)] if chunk > 4 else [(61, 33), (0,), (5,), (7,)]
    local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(3)]
    nbrs[1][0] = nbrs[1][0].astype(np.float64)                       # converted like the single shot
    nbrs[2][0] = np.asfortranarray(nbrs[2][0])                       # non-C-contiguous
    al = [0.25, 0.5, 0.125]
    div = [4.0, 4.0, 4.0] if divide else None
    mx = R.mixer()
    monkeypatch.setattr(R, "NATIVE_PIPELINE", False)
    ref, _ = mx.mix(local, nbrs, al, divisors=div)
    monkeypatch.setattr(R, "NATIVE_PIPELINE", True)
    monkeypatch.setattr(R, "NATIVE_MIN_BYTES", 0)
    got = mx._mix_native(R._layout_of(local), local, nbrs, al, div, chunk_elems=chunk, threads=threads)
    for a, r, s in zip(got, ref, shapes):
        assert a.shape == s and a.dtype == np.float32 and np.array_equal(a, r)
    got2, kept = mx.mix(local, nbrs, al, divisors=div)  # the dispatch takes the native path
    assert kept is None and all(np.array_equal(a, r) for a, r in zip(got2, ref))


def test_hostmixer_native_pipeline_concurrent_threads(gpu):
    """Driver threads (FL_threads_CIFAR100.py runs one per device) calling the native pipeline at
    once: the copy pool serves one call at a time and the others copy on their own thread; every
    result equals its single-threaded one."""
    import threading
    from federated_amd.consensus import _runtime as R
    shapes = [(700, 300), (300,), (300, 40), (40,)]
    jobs = []
    for t in range(6):
        rng = np.random.default_rng(100 + t)
        local = [rng.standard_normal(s).astype(np.float32) for s in shapes]
        nbrs = [[rng.standard_normal(s).astype(np.float32) for s in shapes] for _ in range(2 + t % 3)]
        jobs.append((local, nbrs, [1.0 / (len(nbrs) + 1)] * len(nbrs)))
    mx = R.mixer()
    want = [mx._mix_native(R._layout_of(l), l, nb, al, None, chunk_elems=50_000, threads=1) for l, nb, al in jobs]
    got = [None] * len(jobs)
    errors = []

    def work(i):
        try:
            torch.cuda.set_device(gpu.device)
            l, nb, al = jobs[i]
            for r in range(8):  # helper counts vary between calls and callers (the round-2 deadlock's trigger)
                got[i] = mx._mix_native(R._layout_of(l), l, nb, al, None, chunk_elems=50_000 if r % 2 else 7_777,
                                        threads=(8, 2, 5, 16)[(i + r) % 4])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)
    ths = [threading.Thread(target=work, args=(i,), daemon=True) for i in range(len(jobs))]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=60)
    assert not any(th.is_alive() for th in ths), "a caller did not finish (copy pool stuck?)"
    assert not errors, errors
    for g, w in zip(got, want):
        assert all(np.array_equal(a, b) for a, b in zip(g, w))


def test_bench_shape_round_full_buckets(gpu):
    """The bench workload itself (128 devices x 25M fp32, K = 8 ring window, seeded as bench.py
    seeds them): after one round, the wrap-around devices, the halo-boundary devices and an
    interior one equal the oracle over their whole 25M buckets, bit for bit."""
    from federated_amd.population import RingPopulationShard, RingShardPlan
    L, P, h = 128, 25_000_000, 4
    plan = RingShardPlan(0, 1, L, h)
    shard = RingPopulationShard(plan, P, torch.device("cuda"), None, gpu)
    gen = torch.Generator(device="cuda")
    for i in range(L):
        gen.manual_seed(20261015 + plan.first + i)
        shard.models[i].normal_(generator=gen)
    shard.round()
    torch.cuda.synchronize()
    for i in (0, 3, 4, 64, 123, 127):
        nb = plan.neighbours(i)
        ref = sequential_mix(shard.models[i].cpu().numpy(), [shard.models[j].cpu().numpy() for j in nb], shard.alphas)
        assert np.array_equal(shard.mixed[i].cpu().numpy(), ref), i


@pytest.mark.parametrize("D,hl,hr", [(5, 1, 0), (8, 2, 2), (13, 4, 4), (32, 0, 3), (9, 3, 1)])
@pytest.mark.parametrize("P", [4, 1000, 4100])
def test_ring_round_one_launch_equals_per_device(gpu, D, hl, hr, P):
    """cfa_mix_ring_round_f32 (all window passes of a stacked population in one launch, rows
    derived from base + pitch with ring wrap-around) equals every device's sequential mix with
    its window, bit for bit, for partial last passes and one-sided windows too."""
    g = torch.Generator(device="cuda").manual_seed(D * 1000 + P + 10 * hl + hr)
    models = torch.randn(D, P, device="cuda", generator=g)
    out = torch.full((D, P), float("nan"), device="cuda")
    al = [0.5 / (d + 2) for d in range(D)]
    gpu.ring_round(out, models, torch.tensor(al, dtype=torch.float32, device="cuda"), hl, hr)
    torch.cuda.synchronize()
    h, got = models.cpu().numpy(), out.cpu().numpy()
    for d in range(D):
        nb = [(d + o) % D for o in list(range(-hl, 0)) + list(range(1, hr + 1))]
        assert np.array_equal(got[d], sequential_mix(h[d], [h[j] for j in nb], [al[d]] * len(nb))), d


def test_ring_round_rejects_bad_layouts(gpu):
    from federated_amd import _lib
    m = torch.zeros(4, 1002, device="cuda")
    with pytest.raises(_lib.CFAError, match="16-byte"):
        gpu.ring_round(torch.zeros(4, 1002, device="cuda"), m, torch.zeros(4, device="cuda"), 1, 1)
    m = torch.zeros(4, 1000, device="cuda")
    with pytest.raises(_lib.CFAError, match="wider"):
        gpu.ring_round(torch.zeros(4, 1000, device="cuda"), m, torch.zeros(4, device="cuda"), 2, 2)
    with pytest.raises(_lib.CFAError, match="overlaps"):
        gpu.ring_round(m, m, torch.zeros(4, device="cuda"), 1, 1)


@pytest.mark.parametrize("form", ["compress", "tf1", "tf1_compress", "div"])
def test_hostmixer_zero_copy_equals_staged(gpu, monkeypatch, form):
    """HostMixer.mix's single-shot zero-copy path (kernel on pinned staging) equals the staged
    path (H2D, kernel, D2H) bit for bit, counts included, for every fused form."""
    from federated_amd.consensus import _runtime as R
    rng = np.random.default_rng(5)
    shapes = [(3, 3, 1, 4), (4,), (4096, 6), (6,)]
    local = [(rng.standard_normal(s) * 1e-3).astype(np.float32) for s in shapes]
    nbrs = [[(rng.standard_normal(s) * 1e-3).astype(np.float32) for s in shapes] for _ in range(3)]
    al = [0.25, 0.25, 0.25]
    kw = {}
    if "compress" in form:
        kw["compress"] = (2, 2)
    if form.startswith("tf1"):
        kw["tf1"] = True
    if form == "div":
        kw["divisors"] = [3.0, 3.0, 3.0]
    mx = R.mixer()
    monkeypatch.setattr(R, "SINGLE_ZERO_COPY", False)
    ref, kref = mx.mix(local, nbrs, al, **kw)
    monkeypatch.setattr(R, "SINGLE_ZERO_COPY", True)
    got, kgot = mx.mix(local, nbrs, al, **kw)
    assert kgot == kref
    for a, r in zip(got, ref):
        assert a.dtype == r.dtype and np.array_equal(a, r)


@pytest.mark.parametrize("n,P_odd", [(0, False), (17, False), (3, True), (17, True)])
@pytest.mark.parametrize("form", ["plain", "compress", "tf1", "div"])
def test_hostmixer_zero_copy_edges(gpu, monkeypatch, n, P_odd, form):
    """Zero-copy vs staged equality at the edges the default test misses: no neighbour (the
    C n == 0 branch copies host-mapped memory), n = 17 > CFA_MAX_FANIN (multi-pass with a
    host-resident output) and an odd bucket length (padded pitch)."""
    from federated_amd.consensus import _runtime as R
    if form == "div" and n == 0:
        pytest.skip("the FedAvg form always has at least one model")
    rng = np.random.default_rng(n * 10 + P_odd)
    shapes = [(3, 3, 1, 4), (4,), (257 if P_odd else 256, 6), (7 if P_odd else 6,)]
    local = [(rng.standard_normal(s) * 1e-3).astype(np.float32) for s in shapes]
    nbrs = [[(rng.standard_normal(s) * 1e-3).astype(np.float32) for s in shapes] for _ in range(n)]
    al = [1.0 / (n + 1)] * n
    kw = {"compress": (2, 2)} if form == "compress" else {"tf1": True} if form == "tf1" else {}
    if form == "div":
        kw["divisors"] = [float(j + 2) for j in range(n)]
    mx = R.mixer()
    monkeypatch.setattr(R, "SINGLE_ZERO_COPY", False)
    ref, kref = mx.mix(local, nbrs, al, **kw)
    monkeypatch.setattr(R, "SINGLE_ZERO_COPY", True)
    got, kgot = mx.mix(local, nbrs, al, **kw)
    assert kgot == kref
    for a, r in zip(got, ref):
        assert a.dtype == r.dtype and np.array_equal(a, r)
    if n == 0 and form == "plain":
        for a, x in zip(got, local):
            assert np.array_equal(a, x)


@pytest.mark.parametrize("n,P_odd,compress", [(2, False, None), (2, True, None), (3, True, (2, 2)),
                                              (17, True, None), (1, False, (1, 2))])
@pytest.mark.parametrize("mixed_dtypes", [False, True])
def test_mix_tf1_zero_copy_equals_staged(gpu, monkeypatch, n, P_odd, compress, mixed_dtypes):
    """HostMixer.mix_tf1 (fp64 buckets) with TF1_ZERO_COPY on equals the staged fp64 path bit
    for bit, counts included: odd P (even fp64 pitch), fan-in above CFA_MAX_FANIN, compression,
    and the mixed fp32/fp64 layer runs the reference produces after its first epoch."""
    from federated_amd.consensus import _runtime as R
    rng = np.random.default_rng(n + 100 * P_odd)
    shapes = [(3, 3, 1, 4), (4,), (255 if P_odd else 256, 6), (7 if P_odd else 6,)]

    def model(k):
        dt = np.float64 if (mixed_dtypes and k % 2) else np.float32
        return [(rng.standard_normal(s) * 1e-3).astype(dt) for s in shapes]

    local = model(0)
    nbrs = [model(j + 1) for j in range(n)]
    al = [0.5 / (n + 1)] * n
    mx = R.mixer()
    monkeypatch.setattr(R, "TF1_ZERO_COPY", False)
    ref, kref = mx.mix_tf1(local, nbrs, al, compress=compress)
    monkeypatch.setattr(R, "TF1_ZERO_COPY", True)
    got, kgot = mx.mix_tf1(local, nbrs, al, compress=compress)
    assert kgot == kref
    for a, r in zip(got, ref):
        assert a.dtype == r.dtype and np.array_equal(a, r)


def test_hostmixer_rejects_short_coefficient_lists(gpu, monkeypatch):
    """the zero-copy path calls the C entries directly, which read exactly n
    coefficients; a short alphas or divisors list must raise before any call."""
    from federated_amd.consensus import _runtime as R
    monkeypatch.setattr(R, "SINGLE_ZERO_COPY", True)
    shapes = [(8, 4), (4,)]
    local = [np.ones(s, np.float32) for s in shapes]
    nbrs = [[np.ones(s, np.float32) for s in shapes] for _ in range(3)]
    mx = R.mixer()
    with pytest.raises(ValueError, match="alpha"):
        mx.mix(local, nbrs, [0.25, 0.25])
    with pytest.raises(ValueError, match="divisor"):
        mx.mix(local, nbrs, [0.25] * 3, divisors=[3.0])
    with pytest.raises(ValueError, match="alpha"):
        mx.mix_tf1(local, nbrs, [0.25])
    with pytest.raises(ValueError, match="alpha"):
        mx.mix(local, nbrs, [0.25], tf1=True)


@pytest.mark.parametrize("D,P,u,subset", [(8, 1_071_748, 1.0, False), (32, 24_622, 0.99, True),
                                          (20, 4_000_003, 1.0, False)])
def test_sharded_fedavg_world1_gpu(gpu, D, P, u, subset):
    """ShardedFedAvg on one GPU: the closed-form pre-scaled sum (cfa_mix_f32, all D models in
    one launch chain) equals the reference's sequential FedAvg fold (oracle.ps_fedavg,
    parameter_server_v2.py:159-161) within 1e-5 normwise; world 1 needs no collective."""
    from federated_amd.ps_shard import ShardedFedAvg
    from oracle.cfa_oracle import ps_fedavg
    g = torch.Generator(device="cuda").manual_seed(D + P)
    ps = ShardedFedAvg(0, 1, D, P, "cuda", None, gpu, update_factor=u)
    ps.models.normal_(generator=g)
    ps.params.normal_(generator=g)
    models, params = ps.models.cpu().numpy(), ps.params.cpu().numpy()
    active = [d for d in range(D) if d % 4 != 2] if subset else list(range(D))
    out = ps.aggregate(active).cpu().numpy()
    ref = ps_fedavg([params], [[models[d]] for d in active], u)[0]
    assert np.max(np.abs(out - ref)) <= 1e-5 * np.max(np.abs(ref))


def test_rccl_reduce_sum_world1(gpu):
    """cfa_reduce_sum_f32 through RcclTransport.reduce_sum at world size 1 (identity on root 0)."""
    from federated_amd.dist import RcclTransport
    t = RcclTransport(0, 1, torch.cuda.current_device())
    try:
        x = torch.randn(1 << 20, device="cuda")
        ref = x.clone()
        t.reduce_sum(x, 0)
        t.allreduce_sum(x)
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
    finally:
        t.close()


@pytest.mark.parametrize("rule", [0, 2, 3])
@pytest.mark.parametrize("n,P_odd", [(3, False), (2, True), (17, True)])
def test_fold64_zero_copy_equals_staged(gpu, monkeypatch, rule, n, P_odd):
    """HostMixer.fold64 (the fp64 server-side folds: MQTT PS_server, CFA_FA) on pinned rows in
    place equals the staged H2D / D2H path bit for bit, for every fp64 rule, a payload filler
    neighbour, odd P and fan-in above CFA_MAX_FANIN."""
    from federated_amd import _lib
    from federated_amd.consensus import _runtime as R
    rng = np.random.default_rng(rule * 10 + n)
    shapes = [(5, 7) if P_odd else (4, 8), (3,) if P_odd else (4,)]
    local = [rng.standard_normal(s) for s in shapes]
    nbrs = [[rng.standard_normal(s) for s in shapes] for _ in range(n)]
    flat = np.concatenate([a.reshape(-1) for a in nbrs[-1]])
    nbrs[-1] = lambda dst: np.copyto(dst, flat)  # a payload decoder writes its row itself
    al = [0.9] * n
    div = [float(n)] * n if rule == _lib.RULE_SEQUENTIAL_DIV else None
    mx = R.mixer()
    monkeypatch.setattr(R, "TF1_ZERO_COPY", False)
    ref = mx.fold64(local, nbrs, al, rule, div)
    monkeypatch.setattr(R, "TF1_ZERO_COPY", True)
    got = mx.fold64(local, nbrs, al, rule, div)
    for a, r in zip(got, ref):
        assert a.dtype == np.float64 and np.array_equal(a, r)


@pytest.mark.parametrize("use_filtered,init", [(True, False), (False, False), (False, True)])
@pytest.mark.parametrize("state_dt,grad_dt", [(np.float64, np.float64), (np.float32, np.float32),
                                              (np.float64, np.float32)])
def test_mewma_tf1_zero_copy_equals_staged(gpu, monkeypatch, use_filtered, init, state_dt, grad_dt):
    """HostMixer.mewma_tf1 (CFA-GE) on pinned rows updated in place equals the staged path bit
    for bit: the returned model, and the caller's saved-state arrays at their slots."""
    from federated_amd.consensus import _runtime as R
    rng = np.random.default_rng(7)
    shapes = [(16, 1, 8), (8,), (168, 8), (8,)]
    N, n = 3, 2
    W = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    grads = [[rng.standard_normal(s).astype(grad_dt) for s in shapes] for _ in range(n)]
    st0 = [rng.standard_normal(s + (N,)).astype(state_dt) for s in shapes]
    mx = R.mixer()
    lrs = (0.1, 0.1, 0.2, 0.2)
    s_ref = [x.copy() for x in st0]
    monkeypatch.setattr(R, "TF1_ZERO_COPY", False)
    ref = mx.mewma_tf1(W, s_ref, grads, 0.99, lrs, init, use_filtered)
    s_got = [x.copy() for x in st0]
    monkeypatch.setattr(R, "TF1_ZERO_COPY", True)
    got = mx.mewma_tf1(W, s_got, grads, 0.99, lrs, init, use_filtered)
    for a, r in zip(got, ref):
        assert a.dtype == r.dtype and np.array_equal(a, r)
    for a, r in zip(s_got, s_ref):
        assert a.dtype == r.dtype and np.array_equal(a, r)


@pytest.mark.parametrize("L,hl,hr,C", [(12, 4, 4, 3), (5, 1, 0, 2)])
def test_placement_calibrated_shard_round_equals_oracle(gpu, L, hl, hr, C):
    """A shard whose stacks were chosen by the placement probe (federated_amd/placement.py) mixes
    exactly as the oracle says: the probe changes where the buckets live, not the round; its
    report names one chosen input and one chosen output stack among the candidates."""
    from federated_amd.population import make_ring_shard
    P = 70_001
    shard, info = make_ring_shard(0, 1, L, hl, hr, P, torch.device("cuda"), None, gpu, placement_candidates=C)
    rep = info["placement"]
    assert rep["candidates"] == C and len(rep["in_us"]) == C and len(rep["out_us"]) == C
    assert all(0 <= k < C for k in rep["chosen"]) and all(t > 0 for t in rep["in_us"] + rep["out_us"])
    gen = torch.Generator(device="cuda")
    for i in range(L):
        gen.manual_seed(7 + i)
        shard.models[i].normal_(generator=gen)
    shard.round()
    torch.cuda.synchronize()
    host, mixed = shard.models.cpu().numpy(), shard.mixed.cpu().numpy()
    for i in range(L):
        ref = sequential_mix(host[i], [host[j] for j in shard.plan.neighbours(i)], shard.alphas)
        assert np.array_equal(mixed[i], ref), i
