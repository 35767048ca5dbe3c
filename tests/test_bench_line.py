"""bench.py's driver line: one compact JSON object (< 6 KB) carrying the
contract keys, the roofline / cpu_baseline objects and one-number summaries,
built from a canned full record (tests/golden/bench_full_canned.json, the
shape bench.py writes to its detail side file).  CPU only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CANNED = os.path.join(ROOT, "tests", "golden", "bench_full_canned.json")

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "cpu_baseline_fp32",
            "realtime_streams_per_gpu", "batch1", "batch1_fp32", "batch256", "batch8192", "live", "capacity",
            "capacity_live", "capacity_skewed", "dropin_rt", "detail")
ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic", "roofline_l2", "valu", "binding")
CPU = ("value", "unit", "cores", "kind")


def _line():
    full = json.load(open(CANNED))
    return full, json.dumps(bench.compact_line(full, "gpurun_out/bench_detail.json"), default=bench._json_scalar)


def test_line_is_compact_and_complete():
    full, line = _line()
    assert len(line) < 6000, len(line)
    assert "\n" not in line
    d = json.loads(line)
    for k in REQUIRED:
        assert k in d, k
    for k in ROOF:
        assert k in d["roofline"], k
    for k in CPU:
        assert k in d["cpu_baseline"] and k in d["cpu_baseline_fp32"], k
    # the headline numbers pass through unrounded
    assert d["value"] == full["value"] and d["ms_per_step"] == full["ms_per_step"]
    assert d["roofline"]["frac"] == bench._r(full["roofline"]["frac"])
    # the real-time figure is the tail-criterion live capacity
    assert d["realtime_streams_per_gpu"] == full["capacity_live"]["max_realtime_streams"]
    assert "p99" in d["capacity_live"]["criterion"]
    assert d["capacity"]["criterion"].startswith("throughput ceiling")


def test_line_survives_missing_sections():
    full = json.load(open(CANNED))
    for k in ("batch1", "batch1_fp32", "batch256", "batch8192", "live", "capacity", "capacity_live",
              "capacity_skewed", "cpu_baseline", "cpu_baseline_fp32", "latency", "skewed_int8", "mfma"):
        full.pop(k, None)
    d = json.loads(json.dumps(bench.compact_line(full, None), default=bench._json_scalar))
    assert d["value"] == full["value"] and "roofline" in d and d["detail"] is None


def test_rounding_helper():
    assert bench._r(None) is None
    assert bench._r(456426930.68781596) == 456400000.0
    assert bench._r(0.88216800) == 0.8822


def test_dropin_rt_needs_both_pacings(monkeypatch):
    """dropin_rt counts a thread count as real-time only when its spread and
    burst runs both keep p99 <= 10 ms (canned child outputs, no GPU)."""
    import subprocess
    import types

    def fake_run(cmd, **kw):
        T, mode = int(cmd[1]), cmd[4]
        rt = not (T == 960 and mode == "burst")
        rec = {"threads": T, "frames": 300, "mode": mode, "latency_ms_p50": 1.0, "latency_ms_p99": 2.0 if rt else 12.0,
               "latency_ms_max": 3.0, "deadline_misses": 0, "calls": T * 300, "mean_coalesced_streams": 10.0,
               "realtime_p99": rt}
        return types.SimpleNamespace(stdout=json.dumps(rec) + "\n", returncode=0)

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(os.path, "exists", lambda p: True)
    d = bench.dropin_rt(threads=(256, 960), frames=300)
    assert d["max_threads_realtime_p99"] == 256
    assert d["at_max"]["burst"]["latency_ms_p99"] == 12.0
