"""Metrics printer mirror (printer.rs) and the finish-hook assertion (simulation_callbacks.rs:44-83):
number formatting as serde_json / Rust Display write it, the JSON/table layout, and the printed
values of an engine replica equal to the oracle's on the same scenario."""
import json
import math

import pytest

import parity
import scenarios as sc
from hostcheck_bridge import HostEngine
from kubernetriks_amd import metrics as m


@pytest.mark.parametrize("x,ser,disp", [
    (1.0, "1.0", "1"), (0.5, "0.5", "0.5"), (100.0, "100.0", "100"), (0.1, "0.1", "0.1"),
    (123456.789, "123456.789", "123456.789"), (1e16, "1e16", "10000000000000000"),
    (1.5e-7, "1.5e-7", "0.00000015"), (1e-5, "0.00001", "0.00001"), (1e-6, "1e-6", "0.000001"),
    (2.5e20, "2.5e20", "250000000000000000000"), (-3.25, "-3.25", "-3.25"), (0.0, "0.0", "0"),
    (0.000152, "0.000152", "0.000152"), (4096e-6, "0.004096", "0.004096"),
])
def test_number_formats(x, ser, disp):
    assert m.serde_json_f64(x) == ser
    assert m.rust_display(x) == disp


def test_non_finite_numbers():
    assert m.serde_json_f64(math.nan) == "null" and m.serde_json_f64(math.inf) == "null"
    assert m.rust_display(math.nan) == "NaN" and m.rust_display(math.inf) == "inf"
    assert m.rust_display(-math.inf) == "-inf"


def _engine_and_oracle(scn):
    od, eng = parity.run_pair(HostEngine, scn, log=False)
    assert parity.compare(od, eng, log=False) == []
    return od, eng.results()[0]


def test_metrics_json_layout_and_values():
    od, r = _engine_and_oracle(sc.sc_node_fits_all_pods())
    text = m.assert_and_print(r, "json")
    d = json.loads(text)
    assert list(d) == ["counters", "timings"]
    assert list(d["counters"]) == m.PRINTER_COUNTERS
    assert list(d["timings"]) == ["pod_duration", "pod_schedule_time", "pod_queue_time"]
    for k in m.PRINTER_COUNTERS:
        assert d["counters"][k] == od["counters"][k]
    n, mn, mx, mean, var = od["estimators"]["pod_duration"][:5]
    assert n == 3 and (mn, mx) == (25.0, 100.0)
    assert d["timings"]["pod_duration"] == {"min": mn, "max": mx, "mean": mean, "variance": var}
    assert text.startswith('{\n  "counters": {\n    "total_nodes_in_trace": 1,')
    # printing the oracle's numbers gives the same document
    assert m.metrics_json({"counters": od["counters"], "estimators": od["estimators"]}) == text


def test_metrics_table_layout():
    _, r = _engine_and_oracle(sc.sc_many_pods_one_at_a_time())
    t = m.metrics_table(r)
    lines = t.splitlines()
    assert lines[0].startswith("+") and lines[1].startswith("| Metric") and "| Count" in lines[1]
    assert sum(1 for ln in lines if ln.startswith("| ")) == 11 + 4
    assert "| Pod duration" in t and "| Total pods in trace" in t


def test_empty_estimators_print_null():
    r = {"counters": {k: 0 for k in m.PRINTER_COUNTERS},
         "estimators": {k: [0, math.inf, -math.inf, math.nan, math.nan] for k in
                        ("pod_duration", "pod_schedule_time", "pod_queue_time")}}
    d = json.loads(m.metrics_json(r))
    assert d["timings"]["pod_queue_time"] == {"min": None, "max": None, "mean": None, "variance": None}
    assert "| inf " in m.metrics_table(r) and "NaN" in m.metrics_table(r)


def test_finish_assertion():
    r = {"counters": dict({k: 0 for k in m.PRINTER_COUNTERS}, terminated_pods=2, pods_succeeded=1)}
    with pytest.raises(AssertionError):
        m.assert_and_print(r)


def test_ensemble_summary_pools_estimators():
    s = m.EnsembleSummary(["placements"], ["d"])
    xs = [[1.0, 2.0, 4.0], [8.0], [3.0, 5.0]]
    for part in xs:  # per-replica Welford rows, as the engine keeps them
        n, mean, m2 = 0, 0.0, 0.0
        for x in part:
            n += 1
            dlt = (x - mean) / n
            mean += dlt
            m2 += dlt * dlt * n * (n - 1)
        s.add_replica([len(part)], [[n, min(part), max(part), mean, m2]])
    allx = [x for p in xs for x in p]
    mu = sum(allx) / len(allx)
    t = s.as_dict()["timings"]["d"]
    assert t["n"] == 6 and t["min"] == 1.0 and t["max"] == 8.0
    assert abs(t["mean"] - mu) < 1e-12
    assert abs(t["variance"] - sum((x - mu) ** 2 for x in allx) / 6) < 1e-12
    assert s.as_dict()["counters"]["placements"] == 6


def test_estimator_histograms_count_every_sample_and_match_oracle():
    """K10S_HIST_BINS log2 histograms (engine addition): the oracle's and the engine's agree bin for
    bin (parity.compare checks them), and each holds exactly n samples in the bins the pod
    durations of the reference scenario fall into."""
    import math
    import parity
    import scenarios as sc
    from hostcheck_bridge import HostEngine
    od, eng = parity.run_pair(HostEngine, sc.sc_c1_generic_example(), max_time=20000.0)
    assert parity.compare(od, eng) == []
    est = eng.results()[0]["estimators"]
    for k, row in est.items():
        assert sum(row[5]) == row[0], k
    n, mn, mx = est["pod_duration"][:3]
    lo = 0 if mn < 2 ** -10 else min(31, math.frexp(mn)[1] - 1 + 11)
    hi = 0 if mx < 2 ** -10 else min(31, math.frexp(mx)[1] - 1 + 11)
    h = est["pod_duration"][5]
    assert h[lo] > 0 and h[hi] > 0 and sum(h[lo:hi + 1]) == n


def test_gauge_recorder_rows_and_csv():
    """The 5-s gauge recorder (collector.rs:352-407): engine rows equal the oracle's bit for bit
    (parity.compare), one row per tick from t = 0, and the CSV has the reference's header."""
    import parity
    import scenarios as sc
    from hostcheck_bridge import HostEngine
    from kubernetriks_amd.metrics import GAUGE_COLUMNS, gauge_csv
    od, eng = parity.run_pair(HostEngine, sc.sc_c1_generic_example(), max_time=20000.0)
    assert parity.compare(od, eng) == []
    rows = eng.gauges(0)
    assert len(rows) == len(od["gauges"]) > 0
    assert [r[0] for r in rows[:3]] == [0.0, 5.0, 10.0]
    # 4 pods of 4000 mcpu / 8 GiB on one 16000 mcpu / 16 GiB node: cpu 0.5 (2 pods fit by ram), ram 1.0
    assert (565.0, 1, 4, 4, 0.5, 1.0, 0.5, 1.0) in rows
    text = gauge_csv(rows[113:114])
    assert text.splitlines()[0] == ",".join(GAUGE_COLUMNS)
    assert text.splitlines()[1] == "565,1,4,4,0.5,1,0.5,1"
