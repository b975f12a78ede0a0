"""The bench.py JSON line contract (the driver parses it): one line from rank 0 with the metric BASELINE.json
names, whole-job throughput, the timing fields, `roofline` priced at the bytes the kernel reads (no frac
above 1, the SURVEY 8(d) figure kept apart as a work rate) and `cpu_baseline` from the oracle port.  Runs
the host-check engine (`--selftest-host`: no GPU) on a small C3-shaped cluster; the roofline pricing and
the PMC-traffic lookup are also checked as functions."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _line(args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env, capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_line_carries_the_contract_fields():
    b = _line(["--selftest-host", "--nodes", "64", "--pods", "120", "--arrival-window", "60", "--steps", "2",
               "--warmup", "1", "--replicas", "2", "--cpu-seconds", "1", "--cpu-workers", "2"])
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert b["metric"] == base["metric"]
    assert b["unit"] == "placements/s" and b["higher_is_better"] is True
    assert b["n_gpus"] == 1 and b["steps"] == 2 and b["warmup"] == 1 and b["scaling"] == "weak"
    assert b["value"] > 0 and b["ms_per_step"] > 0 and b["vs_baseline"] is None
    # (on the device the line says "synthetic: ..."; the host self-test names itself instead)
    assert b["dtype"] == "f64" and b["data"].startswith("selftest") and "workload" in b["config"]
    r = b["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0.0 <= r["frac"] <= 1.0   # (the host self-test times no device kernel: 0)
    assert "survey_pricing" in r and "work rate" in r["survey_pricing"]["note"]
    cb = b["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "placements/s" and cb["value"] > 0 and cb["cores"] >= 1
    assert cb["sample"]


def test_roofline_prices_bytes_read():
    import bench
    # 10 attempts over a 100-node cache, 4 placements, 8-B entries, one launch of 1 ms
    r = bench.roofline(8.0, 0.0, scanned=1000, nread=600, attempts=10, placements=4, launches=1, kernel_ms=1.0,
                       traffic=None)
    read = 8.0 * 600 + 12.0 * 10 + 8.0 * 4
    assert abs(r["bytes_per_launch"] - read) < 1e-9
    assert abs(r["achieved"] - read / 1e-3 / 1e9) < 1e-9
    assert abs(r["frac"] - read / 1e-3 / 8e12) < 1e-15
    survey = 12.0 * 1000 + 12.0 * 10 + 12.0 * 4
    assert abs(r["survey_pricing"]["bytes_per_launch"] - survey) < 1e-9
    assert r["traffic"] is None and r["traffic_frac"] is None


def test_pmc_traffic_only_for_the_measured_build():
    import bench
    pm = json.load(open(os.path.join(REPO, "profiles", "pmc_run_kernel.json")))
    R, nodes, pods = pm["config"]
    assert bench.pmc_traffic("c3", R, nodes, pods, False, "least", pm["engine"]) == pm["hbm_bytes_per_launch"]
    assert bench.pmc_traffic("c3", R, nodes, pods, False, "least", pm["engine"] + "x") is None
    assert bench.pmc_traffic("c3", R, nodes, pods // 2, False, "least", pm["engine"]) is None
