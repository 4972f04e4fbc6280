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
    assert rl["job_peak"] == 8000.0 and abs(rl["job_frac"] - d["value"] / 8000.0) < 1e-3
    assert "traffic" in rl
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0 and cb["sample"]
    # value = all algorithmic bytes / time: consistent with ms_per_step
    assert abs(d["value"] - 16 * 10 * 1_000_000 * 4 / (d["ms_per_step"] * 1e-3) / 1e9) <= 0.01 * d["value"]
    # round 6: the headline runs on plain allocations; the calibrated placement is a leg beside it
    assert d["config"]["placement"] is None
    leg = d["legs"]["placement_calibrated"]
    assert leg["value"] > 0 and 0 < leg["frac"] < 1 and leg["placement"]["candidates"] >= 1


N_GT_1_FIELDS = [("value", float), ("ms_per_step", float), ("n_gpus", int), ("exit_status", int),
                 ("config", dict), ("roofline", dict), ("partitions", dict)]
CONFIG_FIELDS = ["partition", "transport", "comparable", "rccl_version", "halo_route", "cache_reuse", "rows_note",
                 "gpus_visible", "ranks_share_gpus", "budget", "headline_fallback", "links", "rccl_log", "host_lane",
                 "halo_check"]


def _self_launched(extra, timeout=240):
    """python3 bench.py --gpus 2 ... with no torch.distributed.run: bench launches its own ranks
    (on a one-GPU box both share the card)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--params", "1000000", "--steps", "3",
           "--warmup", "1", "--no-live-traffic", "--total-seconds", "200"] + extra
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    return r, json.loads(lines[0])


def test_self_launched_n2_line_matches_the_documented_schema():
    """INTEGRATION.md §5 "Fields of the N > 1 line": the devices-partition headline (rehearsed on the
    torch transport, since RCCL refuses two ranks on one device), every documented field present,
    the params leg beside it with its cache-reuse marking, exit status 0."""
    r, d = _self_launched(["--transport", "torch"])
    assert r.returncode == 0, r.stderr[-3000:]
    for key, typ in N_GT_1_FIELDS:
        assert isinstance(d[key], typ), key
    assert d["n_gpus"] == 2 and d["exit_status"] == 0 and d["scaling"] == "strong"
    c = d["config"]
    for key in CONFIG_FIELDS:
        assert key in c, key
    assert c["partition"] == "devices" and c["headline_fallback"] is None
    assert c["transport"] == "torch-gloo" and c["comparable"] is False
    assert set(c["halo_route"]) >= {"relay", "stages", "critical_MB", "autotune", "predicted_critical_ms",
                                    "achieved_critical_ms", "link_cost"}
    # round 5: the link probe's measured rates feed the route plan, and the round is decomposed
    links = c["links"]
    assert links["rates_GBps"][0][1] > 0 and links["rates_GBps"][1][0] > 0 and links["rates_GBps"][0][0] is None
    at = c["halo_route"]["autotune"]
    assert at["mode"] == "links" and at["predicted_ms"] > 0
    assert at["plan"].split("+")[0] in ("uniform", "measured", "direct")
    assert at["candidates_predicted_ms"]["uniform"] > 0 and c["halo_route"]["link_cost"] in ("uniform", "measured")
    # round 6: the ranks run at whatever hardware-queue count the box exports (no override): the
    # lane's waits are on the host, and every stream comes from the rank's stream budget
    import bench
    assert c["gpu_max_hw_queues"] == bench.hw_queues_report(os.environ)
    assert set(c["streams"]["roles"]["0"]) <= {"comm", "lane_out", "lane_in"}
    assert c["host_lane"]["waits"].startswith("host")
    # every halo row the timed rounds delivered equals its owner's row (2 ranks x 8 rows)
    assert c["halo_check"]["rows"] == 16 and c["halo_check"]["mismatches"] == 0
    # the host lane: probed with both ranks on it at once, offered to the plan, reported when used
    hl = c["host_lane"]
    assert len(hl["out_GBps"]) == 2 and min(hl["out_GBps"] + hl["in_GBps"]) > 0
    assert len(hl["topology"]) == 2 and all("pci" in t for t in hl["topology"])
    assert "uniform+lane" in at["candidates_predicted_ms"]
    if at["plan"].endswith("+lane"):
        assert c["halo_route"]["lane"] and c["halo_route"]["lane_MB"] > 0 and at["host_lane"]["in_MB"] > 0
        assert d["decomposition"]["host_lane"]["in_ms"] > 0 and d["decomposition"]["host_lane"]["end_ms"] > 0
    dc = d["decomposition"]
    for key in ("exchange_only_ms", "exchange_groups_ms_sum", "exchange_link_GBps", "exchange_groups",
                "compute_only_ms", "t_mix_ms", "delta", "tail_ms", "model_prediction_ms", "model_simulated_ms",
                "achieved_ms", "bound"):
        assert key in dc, key
    assert dc["exchange_only_ms"] > 0 and dc["compute_only_ms"] > 0 and dc["t_mix_ms"] > 0
    assert len(dc["exchange_groups"]) == c["halo_route"]["groups"]
    assert all(g["ms"] >= 0 and g["busiest_link_MB"] > 0 for g in dc["exchange_groups"])
    assert c["halo_route"]["achieved_critical_ms"] == dc["exchange_groups_ms_sum"]
    assert dc["achieved_ms"] == d["ms_per_step"]
    assert set(c["budget"]) >= {"total_s", "headline_s", "left_s", "skipped"}
    assert d["roofline"]["job_peak"] == 16000.0 and abs(d["roofline"]["job_frac"] - d["value"] / 16000.0) < 1e-3
    # 1M-element rows: a 9-row window fits the Infinity Cache, so the scattered rate is there too
    assert c["cache_reuse"] is True and isinstance(d["value_scattered"], float) and c["rows_note"]
    p = d["partitions"]["params"]
    assert p["cache_reuse"] is True and p["value"] > 0 and p["value_scattered"] > 0
    assert "weak" in d["partitions"]


def test_self_launched_n2_rccl_refused_falls_back_and_exits_3():
    """RCCL cannot open two ranks on one device: the line still comes, with the params headline,
    config.headline_fallback naming the error, the exchanging legs' errors, and status 3."""
    r, d = _self_launched([])
    if d["config"]["headline_fallback"] is None:  # a node where RCCL opened: nothing to check here
        assert r.returncode == 0
        return
    assert r.returncode == 3 and d["exit_status"] == 3
    fb = d["config"]["headline_fallback"]
    assert fb["wanted"] == "devices" and fb["measured"] == "params" and "rccl" in fb["error"]
    assert d["config"]["partition"] == "params" and d["value"] > 0
    assert "error" in d["partitions"]["devices"]


def test_self_launched_headline_failing_on_every_rank_falls_back_and_exits_3():
    """An exchanging headline that raises on every rank (here a hybrid partition whose device groups
    do not divide the world) still yields the line: the params partition measured as the headline,
    the error in config.headline_fallback, status 3."""
    r, d = _self_launched(["--transport", "torch", "--partition", "hybrid", "--device-groups", "3",
                           "--no-extra-legs"])
    assert r.returncode == 3 and d["exit_status"] == 3
    fb = d["config"]["headline_fallback"]
    assert fb["wanted"] == "hybrid" and fb["measured"] == "params" and "dev_groups" in fb["error"]
    assert d["config"]["partition"] == "params" and d["value"] > 0
