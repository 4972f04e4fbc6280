#!/usr/bin/env python3
"""Can a round's halo also travel over PCIe, through pinned host memory, beside xGMI?

At N = 2 the ring halo is 800 MB per rank per round over ONE xGMI link, twice the
interior mixing time; the only other path between two GPUs of a node is each GPU's PCIe link to
host memory (Gen5 x16, 63 GB/s per direction spec). This probe measures what that path gives.

``--mode rates`` (one process): D2H and H2D copy rates between HBM and pinned host memory, each
alone and both at once, at two copy sizes (or those of ``--sweep-mb``); then the headline mix (K = 8 x 25M) alone and while
both copy directions run, which gives the copies' cost to the mixes (delta) and the copy rates
under mixing load.

``--mode xproc`` (parent without GPU + two child processes on the visible GPU): the mechanism
of the host lane across processes. A shared-memory segment per direction, pinned in both
processes with cfa_host_register; each child is the producer of one direction (D2H chunk ->
cfa_stream_signal raises the chunk's sequence number) and the consumer of the other (its host
waits for that number with cfa_host_wait_word, then enqueues the H2D chunk; round 6: no wait on a
GPU queue), two round parities of buffers with an ack word
for back-pressure. Every round the consumer checks the landed rows bit for bit against the
producer's pattern. On a one-GPU box both directions share the one PCIe link, so the rates are
a lower bound for two GPUs.

``--mode probe``: ``linkprobe.probe_lane`` itself, two processes on the GPU, at the message sizes
of ``--sweep-mb`` (default 64, 256, 1024 MB per rank).

Usage (GPU box): python tools/probe/host_lane.py --mode rates [--sweep-mb 2,4,...] | --mode xproc
[--rounds 12] | --mode probe"""
import argparse
import ctypes
import json
import mmap
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

P = 25_000_000
FLAG_BYTES = 4096


def rates(a):
    import torch
    from federated_amd import _lib
    from federated_amd.engine import get_engine
    lib = _lib.load()
    eng = get_engine(0)
    rows = a.rows
    nbytes = rows * P * 4
    dev_src = torch.randn(rows, P, device="cuda")
    dev_dst = torch.empty(rows, P, device="cuda")
    host_a = torch.empty(rows * P, pin_memory=True)
    host_b = torch.empty(rows * P, pin_memory=True)
    host_b.copy_(dev_src.reshape(-1).cpu())
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def d2h(stream, chunk):
        for off in range(0, nbytes, chunk):
            n = min(chunk, nbytes - off)
            _lib.check("memcpy", lib.cfa_memcpy_async(host_a.data_ptr() + off, dev_src.data_ptr() + off, n,
                                                      ctypes.c_void_p(stream.cuda_stream)))

    def h2d(stream, chunk):
        for off in range(0, nbytes, chunk):
            n = min(chunk, nbytes - off)
            _lib.check("memcpy", lib.cfa_memcpy_async(dev_dst.data_ptr() + off, host_b.data_ptr() + off, n,
                                                      ctypes.c_void_p(stream.cuda_stream)))

    def timed(fns, reps=3):
        best = {}
        for _ in range(reps):
            torch.cuda.synchronize()
            evs = []
            for name, f, st in fns:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                f(st)
                e1.record(st)
                evs.append((name, e0, e1))
            torch.cuda.synchronize()
            for name, e0, e1 in evs:
                best[name] = max(best.get(name, 0.0), nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        return {k: round(v, 2) for k, v in best.items()}

    out = {"mode": "rates", "bytes_per_direction": nbytes}
    chunks = [int(c) << 20 for c in a.sweep_mb.split(",")] if a.sweep_mb else [100 << 20, 16 << 20]
    for chunk in chunks:
        tag = f"{chunk >> 20}MB"
        out[f"d2h_alone_{tag}"] = timed([("d2h", lambda s: d2h(s, chunk), s1)])["d2h"]
        out[f"h2d_alone_{tag}"] = timed([("h2d", lambda s: h2d(s, chunk), s2)])["h2d"]
        both = timed([("d2h", lambda s: d2h(s, chunk), s1), ("h2d", lambda s: h2d(s, chunk), s2)])
        out[f"both_{tag}"] = both
    assert torch.equal(dev_dst, dev_src), "H2D landed different bytes"
    # the mix alone and under both copy directions
    K = 8
    ins = torch.randn(K + 1, P, device="cuda")
    mo = torch.empty(P, device="cuda")
    fn = eng.prepare_mix_seq(mo, ins[0], [ins[j] for j in range(1, K + 1)], [1.0 / (K + 1)] * K)
    cs = torch.cuda.current_stream()

    def mixes(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cs)
        for _ in range(n):
            fn(None)
        e1.record(cs)
        return e0, e1

    for _ in range(5):
        fn(None)
    torch.cuda.synchronize()
    e0, e1 = mixes(40)
    torch.cuda.synchronize()
    t_alone = e0.elapsed_time(e1) * 1e3 / 40
    # copies long enough to cover the mixes: rows x 100 MB each way, 3 times
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    c0.record(s1)
    g0.record(s2)
    for _ in range(3):
        d2h(s1, 16 << 20)
        h2d(s2, 16 << 20)
    c1.record(s1)
    g1.record(s2)
    e0, e1 = mixes(40)
    torch.cuda.synchronize()
    t_with = e0.elapsed_time(e1) * 1e3 / 40
    out["mix_alone_us"] = round(t_alone, 2)
    out["mix_with_copies_us"] = round(t_with, 2)
    out["delta"] = round(t_with / t_alone - 1.0, 4)
    out["d2h_under_mix_GBps"] = round(3 * nbytes / (c0.elapsed_time(c1) * 1e-3) / 1e9, 2)
    out["h2d_under_mix_GBps"] = round(3 * nbytes / (g0.elapsed_time(g1) * 1e-3) / 1e9, 2)
    out["mix_window_ms"] = round(e0.elapsed_time(e1), 3)
    out["copy_window_ms"] = round(max(c0.elapsed_time(c1), g0.elapsed_time(g1)), 3)
    print(json.dumps(out), flush=True)


class Segment:
    """One direction's shared segment: [2 parities x chunks x chunk bytes] data + a flag page
    (word 0: ready sequence, word 16: ack sequence, word 32: producer status, word 48: consumer
    status), mapped and pinned in this process."""

    def __init__(self, path, data_bytes, lib):
        from federated_amd import _lib
        self.lib = lib
        fd = os.open(path, os.O_RDWR)
        self.size = data_bytes + FLAG_BYTES
        self.mm = mmap.mmap(fd, self.size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        os.close(fd)
        self.base = ctypes.addressof(ctypes.c_char.from_buffer(self.mm))
        _lib.check("cfa_host_register", lib.cfa_host_register(ctypes.c_void_p(self.base), self.size))
        dp = ctypes.c_void_p()
        _lib.check("cfa_host_device_pointer", lib.cfa_host_device_pointer(ctypes.c_void_p(self.base), ctypes.byref(dp)))
        self.dbase = dp.value
        self.data_bytes = data_bytes

    def word(self, i, dev=True):
        return (self.dbase if dev else self.base) + self.data_bytes + 4 * i

    def read_word(self, i):
        return ctypes.c_uint.from_address(self.word(i, dev=False)).value

    def close(self):
        self.lib.cfa_host_unregister(ctypes.c_void_p(self.base))


def child(a):
    import torch
    from federated_amd import _lib
    lib = _lib.load()
    me = a.child_index
    chunk_elems = a.chunk_mb * (1 << 20) // 4
    rows = a.rows
    total = rows * P
    nch = -(-total // chunk_elems)
    parity_bytes = nch * chunk_elems * 4
    out_seg = Segment(a.seg[me], 2 * parity_bytes, lib)       # I produce into this one
    in_seg = Segment(a.seg[1 - me], 2 * parity_bytes, lib)    # I consume from this one
    g = torch.Generator(device="cuda").manual_seed(1000 + me)
    src = torch.randn(total, device="cuda", generator=g)
    g2 = torch.Generator(device="cuda").manual_seed(1000 + 1 - me)
    expect = torch.randn(total, device="cuda", generator=g2)
    dst = torch.empty(total, device="cuda")
    ps, cs = torch.cuda.Stream(), torch.cuda.Stream()
    psh, csh = ctypes.c_void_p(ps.cuda_stream), ctypes.c_void_p(cs.cuda_stream)
    tmo = int(a.timeout_s * 1e6)
    times, bad = [], 0
    torch.cuda.synchronize()
    for r in range(a.rounds):
        par = r % 2
        # producer: the round's tag in the first element of every chunk, then D2H chunk by chunk
        with torch.cuda.stream(ps):
            src[::chunk_elems] = float(r)
        if r >= 2:  # back-pressure: the consumer has drained round r - 2 from this parity (host wait)
            if lib.cfa_host_wait_word(ctypes.c_void_p(out_seg.word(16, dev=False)), r - 1, tmo) != 0:
                print(json.dumps({"child": me, "round": r, "timeout": "ack"}), flush=True)
                return 3
        for c in range(nch):
            lo = c * chunk_elems
            n = min(chunk_elems, total - lo)
            _lib.check("memcpy", lib.cfa_memcpy_async(ctypes.c_void_p(out_seg.base + par * parity_bytes + lo * 4),
                                                      ctypes.c_void_p(src.data_ptr() + lo * 4), n * 4, psh))
            _lib.check("signal", lib.cfa_stream_signal(ctypes.c_void_p(out_seg.word(0)), r * nch + c + 1, psh))
        # consumer
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cs)
        for c in range(nch):
            lo = c * chunk_elems
            n = min(chunk_elems, total - lo)
            if lib.cfa_host_wait_word(ctypes.c_void_p(in_seg.word(0, dev=False)), r * nch + c + 1, tmo) != 0:
                print(json.dumps({"child": me, "round": r, "timeout": f"chunk {c}"}), flush=True)
                return 3
            _lib.check("memcpy", lib.cfa_memcpy_async(ctypes.c_void_p(dst.data_ptr() + lo * 4),
                                                      ctypes.c_void_p(in_seg.base + par * parity_bytes + lo * 4),
                                                      n * 4, csh))
        _lib.check("signal", lib.cfa_stream_signal(ctypes.c_void_p(in_seg.word(16)), r + 1, csh))
        e1.record(cs)
        cs.synchronize()
        ps.synchronize()
        exp = expect.clone()
        exp[::chunk_elems] = float(r)
        ok = bool(torch.equal(dst, exp))
        bad += not ok
        times.append(e0.elapsed_time(e1))
    nbytes = total * 4
    steady = sorted(times[2:]) or times
    med = steady[len(steady) // 2]
    print(json.dumps({"child": me, "rounds": a.rounds, "bad_rounds": bad, "chunk_MB": a.chunk_mb,
                      "bytes_per_round": nbytes, "round_ms": [round(t, 3) for t in times],
                      "median_GBps": round(nbytes / (med * 1e-3) / 1e9, 2)}), flush=True)
    in_seg.close()
    out_seg.close()
    return 0 if bad == 0 else 4


def xproc(a):
    chunk_elems = a.chunk_mb * (1 << 20) // 4
    total = a.rows * P
    nch = -(-total // chunk_elems)
    data = 2 * nch * chunk_elems * 4
    tag = f"cfa_lane_probe_{os.getpid()}"
    segs = [f"/dev/shm/{tag}_{i}" for i in range(2)]
    st = os.statvfs("/dev/shm")
    info = {"mode": "xproc", "shm_free_GB": round(st.f_bavail * st.f_frsize / 1e9, 2),
            "segment_bytes": data + FLAG_BYTES}
    procs = []
    try:
        for s in segs:
            with open(s, "wb") as f:
                f.truncate(data + FLAG_BYTES)
        cmd = [sys.executable, os.path.abspath(__file__), "--mode", "child", "--rows", str(a.rows),
               "--rounds", str(a.rounds), "--chunk-mb", str(a.chunk_mb), "--timeout-s", str(a.timeout_s),
               "--seg", segs[0], segs[1]]
        procs = [subprocess.Popen(cmd + ["--child-index", str(i)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                  text=True) for i in range(2)]
        deadline = time.monotonic() + a.wall_s
        res = []
        for p in procs:
            try:
                o, e = p.communicate(timeout=max(1.0, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                o, e = p.communicate()
            res.append({"rc": p.returncode, "lines": [json.loads(l) for l in o.splitlines() if l.startswith("{")],
                        "stderr": e[-600:] if p.returncode else ""})
        info["children"] = res
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for s in segs:
            if os.path.exists(s):
                os.unlink(s)
    print(json.dumps(info), flush=True)
    return 0 if all(r["rc"] == 0 for r in info.get("children", [])) else 1


def probe_child(rank, world, port, sizes_mb, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from federated_amd.hostlane import new_token
        from federated_amd.linkprobe import agree_gloo, probe_lane
        out = {}
        for i, mb in enumerate(sizes_mb):
            tok = [new_token() if rank == 0 else None]
            dist.broadcast_object_list(tok, src=0)
            r = probe_lane(rank, world, torch.device("cuda", 0), tok[0], agree_gloo, elems=int(mb * 1e6 / 4),
                           reps=5, timeout_s=15.0)
            out[f"{i}:{mb:g}"] = {"out_GBps": r["out_GBps"], "in_GBps": r["in_GBps"]}  # in call order
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def probe_sizes(a):
    """``linkprobe.probe_lane`` itself (two processes on the GPU, as the N = 2 bench runs it) at
    several message sizes: how far the probed rate depends on the probe's own size."""
    import multiprocessing as mp
    sizes = [float(x) for x in a.sweep_mb.split(",")] if a.sweep_mb else [64.0, 256.0, 1024.0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 35500 + os.getpid() % 997
    procs = [ctx.Process(target=probe_child, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=a.wall_s) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    print(json.dumps({"mode": "probe", "by_size_MB": res[0]}), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["rates", "xproc", "child", "probe"], default="rates")
    ap.add_argument("--rows", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--chunk-mb", type=int, default=16)
    ap.add_argument("--timeout-s", type=float, default=5.0)
    ap.add_argument("--wall-s", type=float, default=150.0)
    ap.add_argument("--sweep-mb", default="", help="rates mode: copy sizes in MB (default 100,16)")
    ap.add_argument("--seg", nargs=2)
    ap.add_argument("--child-index", type=int, default=0)
    a = ap.parse_args()
    if a.mode == "rates":
        return rates(a) or 0
    if a.mode == "child":
        return child(a)
    if a.mode == "probe":
        return probe_sizes(a)
    return xproc(a)


if __name__ == "__main__":
    sys.exit(main())
