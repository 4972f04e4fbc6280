"""Graph-replayed rounds (federated_amd/_graphs.py) equal eager rounds bit for bit.

``PopulationRound.rounds`` and ``CfaGePopulation.rounds`` capture whole periods of their buffer
rotation as hipGraphs. The graphs must hold the same kernels with the same arguments as the
eager rounds, for every starting phase and for round counts that leave partial periods."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D,P,use_window,lists_kind", [(16, 1488, False, "kreg"), (9, 4100, True, "ring"),
                                                      (12, 777, False, "kreg")])
@pytest.mark.parametrize("R", [1, 2, 5, 19])
def test_population_rounds_graph_equals_eager(gpu, D, P, use_window, lists_kind, R):
    from federated_amd import topology as T
    if lists_kind == "kreg":
        lists = T.kregular_v3(D, 2)
    else:  # ring window [d-1, d+1, d+2] (hl 1, hr 2): the window-pass path
        lists = [[(d - 1) % D, (d + 1) % D, (d + 2) % D] for d in range(D)]
    g = torch.Generator(device="cuda").manual_seed(D * 100 + P)
    m0 = torch.randn(D, P, device="cuda", generator=g)
    ref = m0.clone()
    pr_ref = T.PopulationRound(gpu, ref)
    pr_ref.set_topology(lists, T.alphas_tf2, use_window=use_window)
    for _ in range(R):
        pr_ref.run()
        ref.copy_(pr_ref.out)
    got = m0.clone()
    pr = T.PopulationRound(gpu, got)
    pr.set_topology(lists, T.alphas_tf2, use_window=use_window)
    assert (pr.window is not None) == use_window
    out = pr.rounds(R)
    assert out is got
    # a second call starts from the result of the first (reuses the captured graphs)
    pr.rounds(R)
    for _ in range(R):
        pr_ref.run()
        ref.copy_(pr_ref.out)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    eager = m0.clone()
    pe = T.PopulationRound(gpu, eager)
    pe.set_topology(lists, T.alphas_tf2, use_window=use_window)
    pe.rounds(2 * R, graph=False)
    torch.cuda.synchronize()
    assert torch.equal(eager, ref)


def _ge_pop(gpu, ml, D, N, seed):
    from federated_amd import topology
    from federated_amd.cfa_ge_population import CfaGePopulation
    geom = {"filter": 16, "number": 8, "stride": 5} if ml == 1 else {"intermediate_nodes": 32}
    rng = np.random.default_rng(seed)
    B, L, C = 24, 512, 8
    x = torch.from_numpy(rng.standard_normal((D, B, L)).astype(np.float32)).cuda()
    y = torch.from_numpy(np.eye(C, dtype=np.float32)[rng.integers(0, C, (D, B))]).cuda()
    pop = CfaGePopulation(gpu, ml, geom, x, y, topology.kregular_tf1(D, N), 1.0, N, 0.99, 0.1, 0.1)
    W = torch.from_numpy((rng.standard_normal((D, pop.P)) * 0.1).astype(np.float32)).cuda()
    pop.load(W, W.clone())
    return pop


@pytest.mark.parametrize("ml", [1, 2])
@pytest.mark.parametrize("pre,R", [(0, 6), (0, 13), (2, 50), (5, 7)])
def test_cfa_ge_rounds_graph_equals_eager(gpu, ml, pre, R):
    a = _ge_pop(gpu, ml, 16, 2, 7)
    b = _ge_pop(gpu, ml, 16, 2, 7)
    for _ in range(pre):  # start the graph at another phase of the 6-round period
        a.round()
        b.round()
    a.rounds(R, graph=False)
    b.rounds(R)
    b.rounds(3)
    a.rounds(3, graph=False)
    torch.cuda.synchronize()
    for name in ("W", "pub", "S", "G"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name


@pytest.mark.parametrize("pre,R", [(0, 3), (1, 8), (2, 13)])
def test_tf1_population_rounds_graph_equals_eager(gpu, pre, R):
    from federated_amd import topology as T
    D, P = 10, 1488
    g = torch.Generator(device="cuda").manual_seed(77 + pre)
    cur, prev = torch.randn(D, P, device="cuda", generator=g), torch.randn(D, P, device="cuda", generator=g)
    a, b = T.Tf1PopulationRound(gpu, D, P), T.Tf1PopulationRound(gpu, D, P)
    for p in (a, b):
        p.set_topology(T.kregular_tf1(D, 2), T.alphas_tf1_cfa(0.9, 2))
        p.load(cur, prev)
        for _ in range(pre):  # start at another phase of the 3-buffer rotation
            p.round()
    a.rounds(R, graph=False)
    b.rounds(R)
    torch.cuda.synchronize()
    assert torch.equal(a.current, b.current) and torch.equal(a.previous, b.previous)


def test_capture_survives_pending_garbage_strict_mode(gpu):
    """Regression pin for the round-1 abort (commit 99a528c): a dead CUDAGraph and a dead
    torch.cuda.Event sit in a reference cycle, so only the cycle collector can free them. If
    that collection ran mid-capture, it would destroy HIP objects during the capture and abort
    the process. RoundGraphs collects before capturing and pauses the collector while capturing.
    The capture also runs in the strict ("global") mode: after cfa_device_prepare, the launch
    path makes no device query."""
    import gc
    from federated_amd import _graphs
    from federated_amd import topology as T
    assert _graphs.CAPTURE_MODE == "global"

    class Holder:
        pass

    def make_garbage():
        h1, h2 = Holder(), Holder()
        h1.other, h2.other = h2, h1
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.graph(g, stream=s):
            torch.zeros(4, device="cuda").add_(1)
        h1.graph, h2.event = g, torch.cuda.Event()
        h1.event = torch.cuda.Event(enable_timing=True)
        h1.event.record()

    gc.disable()  # keep the cycle alive until the capture's own collection
    try:
        make_garbage()
        assert gc.get_count()[0] > 0
        D, P = 12, 4100
        lists = T.kregular_v3(D, 2)
        m0 = torch.randn(D, P, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
        got = m0.clone()
        pr = T.PopulationRound(gpu, got)
        pr.set_topology(lists, T.alphas_tf2)
        pr.rounds(5)
    finally:
        gc.enable()
    ref = m0.clone()
    pe = T.PopulationRound(gpu, ref)
    pe.set_topology(lists, T.alphas_tf2)
    pe.rounds(5, graph=False)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_tf1_mix_above_fanin_under_capture(gpu):
    """cfa_mix_tf1_f32 with n > CFA_MAX_FANIN chains its passes through an fp64 scratch bucket:
    the engine passes one from torch's allocator (cfa_mix_tf1_ex_f32), so the launch captures
    in the strict mode and replays the eager result bit for bit; the library-allocating entry
    refuses the capture instead of recording an allocation."""
    from federated_amd import _lib
    n, P = 19, 5003
    g = torch.Generator(device="cuda").manual_seed(11)
    local = torch.randn(P, device="cuda", generator=g)
    nbrs = [torch.randn(P, device="cuda", generator=g) for _ in range(n)]
    al = [0.5 / (n + 1)] * n
    ref = torch.empty(P, device="cuda")
    gpu.mix_tf1(ref, local, nbrs, al)
    out = torch.full((P,), float("nan"), device="cuda")
    graph, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(graph, stream=s):
        gpu.mix_tf1(out, local, nbrs, al)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    graph2, s2 = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    s2.wait_stream(torch.cuda.current_stream())
    err = []
    try:
        with torch.cuda.graph(graph2, stream=s2):
            try:
                _lib.call("cfa_mix_tf1_f32", out.data_ptr(), local.data_ptr(),
                          _lib.ptr_table([x.data_ptr() for x in nbrs]), _lib.double_array(al), n, P, 0, 0, 0,
                          None, int(s2.cuda_stream))
            except _lib.CFAError as exc:
                err.append(str(exc))
    finally:
        torch.cuda.synchronize()
    assert err and "graph capture" in err[0]
