"""CPU tests of tools/scale_model.py: the strong-scaling model and its
re-evaluation from measured bench lines (``--from-lines``), with and without the host lane."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "scale_model.py")


def _run(args):
    r = subprocess.run([sys.executable, TOOL] + args, capture_output=True, text=True, timeout=600,
                       env={**os.environ, "PYTHONPATH": ROOT})
    assert r.returncode == 0, r.stderr[-2000:]
    return [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]


def _line(n, ms, value, **cfg):
    return {"n_gpus": n, "ms_per_step": ms, "value": value, "config": cfg.get("config", {}),
            "decomposition": cfg.get("decomposition")}


def test_from_lines_prices_xgmi_and_lane_plans(tmp_path):
    one = _line(1, 19.26, 6646.0)
    xgmi = _line(2, 16.0, 8000.0, config={
        "partition": "devices", "devices_per_gpu": 64, "links": {"median_GBps": 50.0},
        "halo_route": {"critical_MB": 800.0, "lane": False, "autotune": {"predicted_ms": 16.0}}},
        decomposition={"delta": 0.1, "t_mix_ms": 0.15, "tail_ms": 0.3, "model_prediction_ms": 16.3})
    lane = _line(2, 10.8, 11900.0, config={
        "partition": "devices", "devices_per_gpu": 64, "links": {"median_GBps": 50.0},
        "halo_route": {"critical_MB": 400.0, "lane": True, "lane_MB": 800.0, "autotune": {"predicted_ms": 8.4}}},
        decomposition={"delta": 0.1, "t_mix_ms": 0.15, "tail_ms": 0.3, "model_prediction_ms": 10.6})
    f = tmp_path / "lines.jsonl"
    f.write_text("\n".join(json.dumps(x) for x in (one, xgmi, lane)))
    rows = _run(["--from-lines", str(f)])
    assert [r["N"] for r in rows] == [2, 2]
    a, b = rows
    # xGMI only: critical MB over the probed median rate + tail; compute bound 64 x 0.15 x 1.1
    assert a["probe_model_ms"] == round(max(800e6 / 50e9 * 1e3 + 0.3, 64 * 0.15 * 1.1), 4)
    assert "host_lane_MB" not in a
    # with the lane: the kept plan's predicted exchange (link and lane rates) + tail
    assert b["host_lane_MB"] == 800.0
    assert b["probe_model_ms"] == round(max(8.4 + 0.3, 64 * 0.15 * 1.1), 4)
    assert b["achieved_speedup"] == round(11900.0 / 6646.0, 2)


def test_model_table_with_the_lane_at_n2():
    rows = _run(["--t-mix-ms", "0.1502", "--links", "50", "--lane", "0,45", "--delta", "0.1"])
    n2 = next(r for r in rows if r["N"] == 2 and r["partition"] == "devices")
    assert n2["speedup@50GBps,delta0.1"] == 1.18
    assert n2["speedup@50GBps,lane45,delta0.1"] == 1.82 and n2["lane_MB@50GBps,lane45"] > 0
    params = next(r for r in rows if r["N"] == 8 and r["partition"] == "params")
    assert params["speedup@50GBps,lane45,delta0.1"] == 8.0
