"""bench.py's JSON line keeps the driver's contract (one line, the named keys and types), run
as the driver runs it but on a reduced population so it takes seconds."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--params", "1000000", "--devices", "16", "--steps", "3",
           "--warmup", "1", "--cpu-seconds", "0.5", "--cpu-pool-seconds", "0", "--no-live-traffic"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for key, typ in [("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int),
                     ("warmup", int), ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str),
                     ("dtype", str), ("data", str), ("config", dict), ("roofline", dict), ("cpu_baseline", dict)]:
        assert isinstance(d[key], typ), key
    assert d["metric"] == "device-resident GB/s, CFA reduce of K neighbour fp32 param buckets; 1/2/4/8 GPU"
    assert d["unit"] == "GB/s" and d["n_gpus"] == 1 and d["steps"] == 3 and d["higher_is_better"] is True
    assert d["scaling"] in ("strong", "weak") and d["vs_baseline"] is None
    assert "workload" in d["config"]
    rl = d["roofline"]
    assert rl["bound"] == "hbm" and rl["unit"] == "GB/s" and rl["peak"] == 8000.0
    assert 0 < rl["frac"] < 1 and abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-3
    assert "traffic" in rl
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0 and cb["sample"]
    # value = all algorithmic bytes / time: consistent with ms_per_step
    assert abs(d["value"] - 16 * 10 * 1_000_000 * 4 / (d["ms_per_step"] * 1e-3) / 1e9) <= 0.01 * d["value"]
