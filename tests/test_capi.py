"""CPU checks of the C-ABI boundary: libcfa.so loads, exports every symbol include/cfa_engine.h
declares, and the ctypes table matches the header one for one. No compute calls (no GPU)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "cfa_engine.h")


def _header_text():
    with open(HEADER) as fh:
        return fh.read()


def header_symbols():
    text = _header_text()
    return sorted(set(re.findall(r"CFA_API\s+[\w\s\*]+?\b(cfa_\w+)\s*\(", text)))


def test_header_declares_full_abi():
    syms = header_symbols()
    for required in ("cfa_mix_seq_f32", "cfa_mix_f32", "cfa_mewma_update_f32",
                     "cfa_compress_epilogue_f32", "cfa_mix_population_f32", "cfa_comm_init",
                     "cfa_halo_exchange_f32", "cfa_allreduce_sum_f32", "cfa_last_error", "cfa_version"):
        assert required in syms


def test_library_exports_every_header_symbol():
    from federated_amd import _lib
    lib = _lib.load()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\sT\s+(cfa_\w+)", out))
    assert set(header_symbols()) <= exported
    # ... and nothing else: measurement-only kernels live in libcfa_exp.so, not in the product
    assert exported == set(header_symbols()), sorted(exported - set(header_symbols()))
    for name in header_symbols():
        assert hasattr(lib, name)


def test_ctypes_table_matches_header():
    from federated_amd import _lib
    assert sorted(_lib.SIGNATURES) == header_symbols()
    text = _header_text()
    for name, (_, args) in _lib.SIGNATURES.items():
        m = re.search(r"CFA_API[^;(]*\b%s\s*\(([^)]*)\)" % name, text, re.S)
        decl = m.group(1).strip()
        nargs = 0 if decl in ("", "void") else decl.count(",") + 1
        assert nargs == len(args), name


def test_version_and_error_calls_without_gpu():
    from federated_amd import _lib
    lib = _lib.load()
    assert lib.cfa_version() == 10000
    assert isinstance(lib.cfa_last_error(), bytes)


def test_invalid_arguments_fail_loudly_before_any_device_work():
    """Argument validation runs on the host: a bad call returns CFA_E_INVALID and the shim
    raises with the library's message (no device touched for these)."""
    from federated_amd import _lib
    with pytest.raises(_lib.CFAError, match="negative fan-in"):
        _lib.call("cfa_mix_seq_f32", 1 << 20, 1 << 20, None, _lib.float_array([0.5]), -1, 16, None)
    with pytest.raises(_lib.CFAError, match="unknown compression mode"):
        _lib.call("cfa_compress_epilogue_f32", 1 << 20, None, 9, 16, 1 << 21, None)
    with pytest.raises(_lib.CFAError, match="null communicator"):
        _lib.call("cfa_allreduce_sum_f32", None, None, None, 4, None)


def test_wait_signal_sees_a_word_set_by_another_thread_without_gpu():
    """cfa_wait_signal returns as soon as its host word holds the value (acquire loads): here a
    host thread stores it after 20 ms, inside the spin budget, so no HIP call is made. A null
    word fails before anything else."""
    import ctypes
    import threading
    import time

    from federated_amd import _lib
    lib = _lib.load()
    word = (ctypes.c_uint * 1)(0)
    addr = ctypes.addressof(word)

    def setter():
        time.sleep(0.02)
        word[0] = 7

    th = threading.Thread(target=setter)
    t0 = time.perf_counter()
    th.start()
    rc = lib.cfa_wait_signal(addr, 7, None, 10_000_000)  # 10 s spin budget: never reached
    th.join()
    assert rc == 0 and word[0] == 7
    assert time.perf_counter() - t0 < 5.0
    assert lib.cfa_wait_signal(addr, 7, None, 0) == 0  # already set: returns on the first load
    with pytest.raises(_lib.CFAError, match="null signal word"):
        _lib.call("cfa_wait_signal", None, 1, None, 0)
    with pytest.raises(_lib.CFAError, match="null signal word"):
        _lib.call("cfa_stream_signal", None, 1, None)


def test_host_lane_entry_points_validate_before_any_hip_call():
    """The host lane's C-ABI refuses null words / ranges and a non-positive timeout before it
    touches HIP (no GPU here)."""
    import ctypes

    from federated_amd import _lib
    word = (ctypes.c_uint * 2)(0, 0)
    addr = ctypes.addressof(word)
    with pytest.raises(_lib.CFAError, match="null wait word"):
        _lib.call("cfa_host_wait_word", None, 1, 1000)
    with pytest.raises(_lib.CFAError, match="timeout_us must be positive"):
        _lib.call("cfa_host_wait_word", addr, 1, 0)
    with pytest.raises(_lib.CFAError, match="null or empty host range"):
        _lib.call("cfa_host_register", None, 4096)
    with pytest.raises(_lib.CFAError, match="null or empty host range"):
        _lib.call("cfa_host_register", addr, 0)
    with pytest.raises(_lib.CFAError, match="null host pointer"):
        _lib.call("cfa_host_unregister", None)


def test_host_wait_word_release_timeout_and_wrap():
    """cfa_host_wait_word (the host lane's receive-side wait, host only): returns once another
    thread raises the word, in sequence order (a later value also releases it, across the 32-bit
    wrap); gives up with CFA_E_TIMEOUT after its timeout; several threads may wait at once (no
    process-wide state)."""
    import ctypes
    import threading
    import time

    from federated_amd import _lib
    lib = _lib.load()
    words = (ctypes.c_uint * 4)(0, 0, 0xFFFFFFFE, 0)
    addr = ctypes.addressof(words)

    def setter(i, v, delay):
        time.sleep(delay)
        words[i] = v

    th = [threading.Thread(target=setter, args=(0, 9, 0.03)), threading.Thread(target=setter, args=(1, 4, 0.05))]
    rcs = {}

    def waiter(i, v):
        rcs[i] = lib.cfa_host_wait_word(addr + 4 * i, v, 10_000_000)
    ws = [threading.Thread(target=waiter, args=(0, 7)), threading.Thread(target=waiter, args=(1, 4))]
    t0 = time.perf_counter()
    for t in ws + th:
        t.start()
    for t in ws + th:
        t.join()
    assert rcs == {0: 0, 1: 0} and time.perf_counter() - t0 < 5.0  # 9 >= 7 in sequence order
    words[2] = 3  # wrapped past 0xFFFFFFFE: 3 is "after" 0xFFFFFFFF
    assert lib.cfa_host_wait_word(addr + 8, 0xFFFFFFFF, 1000) == 0
    t0 = time.perf_counter()
    rc = lib.cfa_host_wait_word(addr + 12, 1, 100_000)  # never raised
    dt = time.perf_counter() - t0
    assert rc == _lib.CFA_E_TIMEOUT and 0.09 < dt < 3.0
    assert b"expected 1" in lib.cfa_last_error()


def test_single_hip_runtime_in_process():
    """libcfa must bind to the HIP runtime torch loaded (one libamdhip64 mapped)."""
    import torch  # noqa: F401
    from federated_amd import _lib
    _lib.load()
    assert len(_lib.loaded_hip_runtimes()) == 1, _lib.loaded_hip_runtimes()


def test_product_has_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from federated_amd.engine import get_engine
    with pytest.raises(RuntimeError, match="no ROCm GPU"):
        get_engine()


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "federated_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, re.M), f


# SURVEY.md §8(b) "New C-ABI the shim must export": the sketched parameter lists (names only, in
# order). None = the sketch elides the parameters ("(...)"); the entries it names but the library
# does not provide map to None with the reason in the header's departures list.
SKETCH_8B = {
    "cfa_mix_f32": ["out", "local", "nbrs", "n", "coeff", "P", "hip_stream"],
    "cfa_mix_strided_f32": None,  # sketched as "(..., nbr_stride)"; not provided
    "cfa_mewma_update_f32": ["W", "s", "g", "n", "rho", "lr", "use_filtered", "P", "stream"],
    "cfa_compress_epilogue_f32": ["y", "ref_or_null", "thr", "rep", "mode", "kept_count", "P", "stream"],
    "cfa_mix_population_f32": ["out_stack", "in_stack", "csr_ptr", "csr_idx", "csr_coeff", "D", "P", "stream"],
    "cfa_comm_init": ["rank", "nranks", "nccl_unique_id", "comm"],
    "cfa_halo_exchange_f32": None,
    "cfa_allreduce_scaled_f32": None,  # became cfa_allreduce_sum_f32 / cfa_reduce_sum_f32
    "cfa_comm_destroy": ["comm"],
    "cfa_last_error": [],
    "cfa_version": [],
}

# The library's parameter lists for the same entries (what include/cfa_engine.h must declare).
ABI_8B = {
    "cfa_mix_f32": ["out", "local", "nbrs", "coeff", "n", "P", "stream"],
    "cfa_mewma_update_f32": ["W", "s", "g", "g_stride", "n", "rho", "lr1", "lr2", "lr_split", "init",
                             "use_filtered", "P", "stream"],
    "cfa_compress_epilogue_f32": ["y", "ref", "mode", "P", "kept_count", "stream"],
    "cfa_mix_population_f32": ["out_ptrs", "src_ptrs", "csr_ptr", "csr_idx", "csr_coef", "D", "rule", "P",
                               "stream"],
    "cfa_comm_init": ["comm", "rank", "nranks", "id", "device"],
    "cfa_halo_exchange_f32": ["comm", "send_bufs", "send_peers", "nsend", "recv_bufs", "recv_peers", "nrecv",
                              "P", "stream"],
    "cfa_comm_destroy": ["comm"],
    "cfa_last_error": [],
    "cfa_version": [],
}

# Names the sketch and the ABI give the same parameter.
_SAME = {"hip_stream": "stream", "nccl_unique_id": "id", "ref_or_null": "ref", "csr_coeff": "csr_coef"}


def _prototype_params(name):
    m = re.search(r"CFA_API[^;(]*\b%s\s*\(([^)]*)\)\s*;" % name, _header_text(), re.S)
    assert m, name
    decl = " ".join(m.group(1).split())
    if decl in ("", "void"):
        return []
    return [re.findall(r"(\w+)\s*$", p.strip())[0] for p in decl.split(",")]


def _departures():
    text = _header_text()
    start = text.index("Where the ABI departs from the signatures sketched")
    return text[start:text.index("*/", start)]


@pytest.mark.parametrize("name", sorted(ABI_8B))
def test_prototype_parameter_order_against_survey_8b(name):
    """Every entry SURVEY §8(b) sketches: the header's prototype has exactly the parameter order of
    ABI_8B, and where that order differs from the sketch (beyond a renamed parameter) the entry is
    named in the header's departures list, with every sketch parameter it drops or moves."""
    got = _prototype_params(name)
    assert got == ABI_8B[name], (name, got)
    sketch = SKETCH_8B[name]
    norm = [_SAME.get(p, p) for p in sketch] if sketch is not None else None
    deps = _departures()
    if norm is None or norm != got:
        assert re.search(r"- %s\b" % name, deps) or name in deps, f"{name} departs from §8(b) silently"
    if norm is not None and norm != got:
        # the departure text names the entry's own full parameter list, in order
        assert "%s(%s)" % (name, ", ".join(got)) in " ".join(deps.replace("*", " ").split()), name


def test_sketched_entries_not_provided_are_explained():
    exported = set(header_symbols())
    deps = _departures()
    for name, params in SKETCH_8B.items():
        if name not in exported:
            assert name in deps, f"{name} (sketched in SURVEY §8(b)) is neither exported nor explained"


def test_mix_f32_swap_is_stated():
    """Round-4 review: the header claimed cfa_mix_f32 was 'as sketched' while it swaps n and coeff."""
    deps = " ".join(_departures().replace("*", " ").split())
    assert "SWAPPED" in deps and "(out, local, nbrs, n, coeff, P, stream)" in deps


def test_lane_pump_host_mode_walks_waits_copies_signals_and_marks():
    """cfa_lane_pump_* in host mode (no GPU): a round of three operations. The first waits for a word
    another thread raises later and copies; its mark is published only then (a wait for mark 2 is
    still pending before); the last raises the ack word. A round whose word never comes ends with
    CFA_E_TIMEOUT, which is then sticky for waits and submits; destroy interrupts a pending wait."""
    import ctypes
    import threading
    import time

    from federated_amd import _lib
    lib = _lib.load()
    words = (ctypes.c_uint * 4)(0, 0, 0, 0)
    waddr = ctypes.addressof(words)
    src = (ctypes.c_float * 8)(*range(8))
    dst = (ctypes.c_float * 8)()
    pump = ctypes.c_void_p()
    _lib.check("create", lib.cfa_lane_pump_create(ctypes.byref(pump), None, 0, 1))
    ops = (_lib.LaneOp * 3)(
        _lib.LaneOp(wait_word=waddr, wait_value=5, dst=ctypes.addressof(dst), src=ctypes.addressof(src), bytes=16,
                    mark=1),
        _lib.LaneOp(wait_word=waddr, wait_value=6, dst=ctypes.addressof(dst) + 16, src=ctypes.addressof(src) + 16,
                    bytes=16, mark=2),
        _lib.LaneOp(signal_word=waddr + 4, signal_value=9))
    _lib.check("submit", lib.cfa_lane_pump_submit(pump, ctypes.cast(ops, ctypes.c_void_p), 3, 5_000_000))
    assert lib.cfa_lane_pump_submit(pump, ctypes.cast(ops, ctypes.c_void_p), 3, 5_000_000) == _lib.CFA_E_INVALID
    assert lib.cfa_lane_pump_wait(pump, 1, 50_000) == _lib.CFA_E_TIMEOUT  # word 0 still 0: not yet
    words[0] = 5
    assert lib.cfa_lane_pump_wait(pump, 1, 5_000_000) == 0 and list(dst[:4]) == [0.0, 1.0, 2.0, 3.0]
    assert lib.cfa_lane_pump_wait(pump, 2, 50_000) == _lib.CFA_E_TIMEOUT
    threading.Timer(0.05, lambda: words.__setitem__(0, 6)).start()
    assert lib.cfa_lane_pump_wait(pump, -1, 5_000_000) == 0
    assert list(dst[4:]) == [4.0, 5.0, 6.0, 7.0] and words[1] == 9
    # a round whose word never comes: the pump's own wait times out after 0.1 s, sticky
    bad = (_lib.LaneOp * 1)(_lib.LaneOp(wait_word=waddr + 8, wait_value=1, mark=1))
    _lib.check("submit", lib.cfa_lane_pump_submit(pump, ctypes.cast(bad, ctypes.c_void_p), 1, 100_000))
    t0 = time.perf_counter()
    assert lib.cfa_lane_pump_wait(pump, -1, 5_000_000) == _lib.CFA_E_TIMEOUT
    assert 0.08 < time.perf_counter() - t0 < 3.0 and b"timed out" in lib.cfa_last_error()
    assert lib.cfa_lane_pump_wait(pump, 1, 1000) == _lib.CFA_E_TIMEOUT
    assert lib.cfa_lane_pump_submit(pump, ctypes.cast(ops, ctypes.c_void_p), 3, 5_000_000) == _lib.CFA_E_TIMEOUT
    assert lib.cfa_lane_pump_destroy(pump) == 0
    # destroy while a wait is pending (60 s timeout): returns promptly
    p2 = ctypes.c_void_p()
    _lib.check("create", lib.cfa_lane_pump_create(ctypes.byref(p2), None, 0, 1))
    _lib.check("submit", lib.cfa_lane_pump_submit(p2, ctypes.cast(bad, ctypes.c_void_p), 1, 60_000_000))
    time.sleep(0.02)
    t0 = time.perf_counter()
    assert lib.cfa_lane_pump_destroy(p2) == 0 and time.perf_counter() - t0 < 2.0
    with pytest.raises(_lib.CFAError, match="timeout_us must be positive"):
        _lib.call("cfa_lane_pump_wait", ctypes.c_void_p(1), 1, 0)
    with pytest.raises(_lib.CFAError, match="null pump"):
        _lib.call("cfa_lane_pump_submit", None, None, 0, 1)
