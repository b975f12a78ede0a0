"""Metrics output of one replica, and the cross-replica (cross-rank) ensemble summary.

Per replica this mirrors the reference's metrics printer (`src/metrics/printer.rs`):
  * `metrics_json(result)`   = `print_metrics_as_json` (printer.rs:118-164): serde_json
    `to_string_pretty` of `{counters: {10 u64}, timings: {pod_duration, pod_schedule_time,
    pod_queue_time: {min, max, mean, variance}}}`; non-finite floats serialize as `null` like
    serde_json does.
  * `metrics_table(result)`  = `print_metrics_as_pretty_table` (printer.rs:27-81): the two
    prettytable-rs tables (FORMAT_DEFAULT: `|` borders, `-`/`+` separators between every row),
    floats in Rust `Display` form.
  * `assert_and_print(result, fmt)` = the finish hook of RunUntilAllPodsAreFinishedCallbacks
    (simulation_callbacks.rs:44-83): the terminated-pods identity, then the printer.
The estimator values are the engine's own per-replica `average` 0.15 restatements (`collector.rs:15-74`,
DESIGN.md §4), read back bit-exactly; nothing here recomputes them.

Across replicas there is no reference counterpart: `EnsembleSummary` sums the
u64 counters and merges the per-replica estimators in global replica order (Chan et al. pairwise
update of (n, mean, M2), min/max), so the summary of R replicas is bit-identical whether they ran
on one GPU or were sharded over several ranks (`kubernetriks_amd/ensemble.py` gathers them in rank
order before merging).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

PRINTER_COUNTERS = [  # printer.rs:90-101, in declaration (= serialization) order
    "total_nodes_in_trace", "total_pods_in_trace", "pods_succeeded", "pods_unschedulable", "pods_failed",
    "pods_removed", "total_scaled_up_nodes", "total_scaled_down_nodes", "total_scaled_up_pods",
    "total_scaled_down_pods",
]
TIMINGS = [  # printer.rs:104-108 field name -> engine estimator name
    ("pod_duration", "pod_duration"),
    ("pod_schedule_time", "pod_schedule_time"),
    ("pod_queue_time", "pod_queue_time"),
]
TABLE_COUNTER_LABELS = [  # printer.rs:36-51
    "Total nodes in trace", "Total pods in trace", "Pods succeeded", "Pods unschedulable", "Pods failed",
    "Pods removed", "Total scaled up nodes", "Total scaled down nodes", "Total scaled up pods",
    "Total scaled down pods",
]
TABLE_TIMING_LABELS = ["Pod duration", "Pod schedule time", "Pod queue time"]  # printer.rs:56-77


# ---- float formatting -----------------------------------------------------------------------------
def _digits(x: float):
    """Shortest round-trip decimal digits of a finite positive double and the position of the
    decimal point: x = 0.<digits> * 10^point."""
    r = repr(x).lower()
    if "e" in r:
        mant, ex = r.split("e")
        ex = int(ex)
    else:
        mant, ex = r, 0
    ip, _, fp = mant.partition(".")
    alld = ip + fp
    stripped = alld.lstrip("0")
    point = len(ip) - (len(alld) - len(stripped)) + ex
    return stripped.rstrip("0") or "0", point


def rust_display(x: float) -> str:
    """Rust `impl Display for f64` (`{}`): shortest round-trip digits, never an exponent,
    `inf`/`-inf`/`NaN`, integral values without a fractional part (1.0 -> "1")."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    if x == 0.0:
        return "-0" if math.copysign(1.0, x) < 0 else "0"
    sign = "-" if x < 0 else ""
    digits, point = _digits(abs(x))
    if point <= 0:
        s = "0." + "0" * (-point) + digits
    elif point >= len(digits):
        s = digits + "0" * (point - len(digits))
    else:
        s = digits[:point] + "." + digits[point:]
    return sign + s


def serde_json_f64(x: float) -> str:
    """serde_json's f64 serialization (ryu `format64`): non-finite -> `null`; integral values keep
    `.0`; plain decimal for exponents in [-5, 16), otherwise `<d>.<ddd>e<exp>`."""
    if math.isnan(x) or math.isinf(x):
        return "null"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    digits, k = _digits(abs(x))  # value = 0.<digits> * 10^k
    n = len(digits)
    if 0 < k <= 16:
        if n <= k:
            return sign + digits + "0" * (k - n) + ".0"
        return sign + digits[:k] + "." + digits[k:]
    if -5 < k <= 0:
        return sign + "0." + "0" * (-k) + digits
    mant = digits[0] + ("." + digits[1:] if n > 1 else "")
    return sign + mant + "e" + str(k - 1)


# ---- printer.rs restatements ----------------------------------------------------------------------
def _timing_values(result: dict, est_name: str):
    _, mn, mx, mean, var = result["estimators"][est_name][:5]
    return mn, mx, mean, var


def metrics_json(result: dict) -> str:
    """printer.rs:118-164 (`serde_json::to_string_pretty`: 2-space indent, declaration order)."""
    c = result["counters"]
    lines = ["{", '  "counters": {']
    for i, k in enumerate(PRINTER_COUNTERS):
        lines.append(f'    "{k}": {int(c[k])}' + ("," if i + 1 < len(PRINTER_COUNTERS) else ""))
    lines += ["  },", '  "timings": {']
    for j, (field_name, est) in enumerate(TIMINGS):
        mn, mx, mean, var = _timing_values(result, est)
        lines.append(f'    "{field_name}": {{')
        vals = [("min", mn), ("max", mx), ("mean", mean), ("variance", var)]
        for i, (k, v) in enumerate(vals):
            lines.append(f'      "{k}": {serde_json_f64(v)}' + ("," if i + 1 < len(vals) else ""))
        lines.append("    }" + ("," if j + 1 < len(TIMINGS) else ""))
    lines += ["  }", "}"]
    return "\n".join(lines)


def _table(rows: List[List[str]]) -> str:
    """prettytable-rs FORMAT_DEFAULT: padding 1, `|` column separators and borders, a `+---+` line
    above, below and between every pair of rows, left-aligned cells."""
    ncol = max(len(r) for r in rows)
    width = [0] * ncol
    for r in rows:
        for i, cell in enumerate(r):
            width[i] = max(width[i], len(cell))
    sep = "+" + "+".join("-" * (w + 2) for w in width) + "+"
    out = [sep]
    for r in rows:
        cells = [(r[i] if i < len(r) else "") for i in range(ncol)]
        out.append("|" + "|".join(" " + cells[i].ljust(width[i]) + " " for i in range(ncol)) + "|")
        out.append(sep)
    return "\n".join(out) + "\n"


def metrics_table(result: dict) -> str:
    """printer.rs:27-81 (the aggregated counters table, then the stats table)."""
    c = result["counters"]
    agg = [["Metric", "Count"]] + [[lab, str(int(c[k]))] for lab, k in zip(TABLE_COUNTER_LABELS, PRINTER_COUNTERS)]
    stats = [["Metric", "Min", "Max", "Mean", "Variance"]]
    for lab, (_, est) in zip(TABLE_TIMING_LABELS, TIMINGS):
        stats.append([lab] + [rust_display(v) for v in _timing_values(result, est)])
    return _table(agg) + _table(stats)


def assert_and_print(result: dict, fmt: str = "json") -> str:
    """simulation_callbacks.rs:44-83: terminated == succeeded + unschedulable + failed + removed
    (assert_eq!, a panic in the reference), then the printer output (printer.rs:20-25)."""
    c = result["counters"]
    total = c["pods_succeeded"] + c["pods_unschedulable"] + c["pods_failed"] + c["pods_removed"]
    if c["terminated_pods"] != total:
        raise AssertionError(f"terminated_pods {c['terminated_pods']} != {total}")
    return metrics_json(result) if fmt == "json" else metrics_table(result)


# ---- gauge recorder CSV (collector.rs:215-226 header, 392-407 rows) -----------------------------
GAUGE_COLUMNS = ["timestamp", "current_nodes", "current_pods", "pods_in_scheduling_queues",
                 "node_average_cpu_utilization", "node_average_ram_utilization",
                 "cluster_total_cpu_utilization", "cluster_total_ram_utilization"]


def gauge_csv(rows) -> str:
    """experiments/gauge_metrics.csv as the reference writes it (csv crate, `to_string()` of each
    value: Rust Display for f64, decimal for u64) from Engine.gauges() rows."""
    out = [",".join(GAUGE_COLUMNS)]
    for r in rows:
        out.append(",".join([rust_display(float(r[0]))] + [str(int(v)) for v in r[1:4]] +
                            [rust_display(float(v)) for v in r[4:8]]))
    return "\n".join(out) + "\n"


# ---- cross-replica summary ----------------------------------------------------
class EnsembleSummary:
    """Counters summed over replicas; estimators merged in the order replicas are added.

    Each per-replica estimator enters as (n, min, max, mean, M2) with M2 = n * population_variance
    (the engine's `sum2`).  Merging (na, ma, Ma) with (nb, mb, Mb): n = na + nb, d = mb - ma,
    mean = ma + d * nb / n, M2 = Ma + Mb + d^2 * na * nb / n (Chan, Golub, LeVeque 1979)."""

    def __init__(self, counter_names: Sequence[str], est_names: Sequence[str]):
        self.counter_names = list(counter_names)
        self.est_names = list(est_names)
        self.counters = [0] * len(self.counter_names)
        self.est = {k: [0, math.inf, -math.inf, 0.0, 0.0] for k in self.est_names}
        self.replicas = 0
        self.status: Dict[str, int] = {}
        self.hist = None  # {est name: [counts per log2 bin]} once set_histograms() ran

    def add_replica(self, counters: Sequence[int], est_rows: Sequence[Sequence[float]], status: str = "finished"):
        for i, v in enumerate(counters):
            self.counters[i] += int(v)
        for k, row in zip(self.est_names, est_rows):
            self._merge(k, row)
        self.replicas += 1
        self.status[status] = self.status.get(status, 0) + 1

    def _merge(self, k: str, row):
        nb = int(row[0])
        if nb == 0:
            return
        mnb, mxb, mb, m2b = float(row[1]), float(row[2]), float(row[3]), float(row[4])
        a = self.est[k]
        na = a[0]
        if na == 0:
            self.est[k] = [nb, mnb, mxb, mb, m2b]
            return
        n = na + nb
        d = mb - a[3]
        a[3] = a[3] + d * (float(nb) / float(n))
        a[4] = a[4] + m2b + d * d * (float(na) * float(nb) / float(n))
        a[0] = n
        a[1] = min(a[1], mnb)
        a[2] = max(a[2], mxb)

    def set_histograms(self, hist):
        """hist: rows of K10S_HIST_BINS counts per estimator (summed over the job's replicas)."""
        self.hist = {k: [int(v) for v in row] for k, row in zip(self.est_names, hist)}

    def as_dict(self) -> dict:
        out = {"replicas": self.replicas, "replica_status": dict(self.status),
               "counters": {k: v for k, v in zip(self.counter_names, self.counters)}, "timings": {}}
        for k in self.est_names:
            n, mn, mx, mean, m2 = self.est[k]
            out["timings"][k] = {"n": n, "min": mn if n else math.nan, "max": mx if n else math.nan,
                                 "mean": mean if n else math.nan, "variance": (m2 / n) if n else math.nan}
        if self.hist is not None:
            # bin 0: < 2^-10 s; bin k: [2^(k-11), 2^(k-10)) s; last bin: >= 2^20 s
            out["histograms"] = {"log2_lower_edge_s": [None] + list(range(-10, 21)), **self.hist}
        return out


def estimator_rows(raw_result) -> List[List[float]]:
    """(n, min, max, mean, M2) rows of one engine ReplicaResult (ctypes); M2 is the engine's sum2."""
    return [[float(e.n), e.min, e.max, e.mean, e.sum2] for e in raw_result.est]
