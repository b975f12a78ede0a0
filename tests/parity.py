"""Engine-vs-oracle comparison used by the parity tests (CPU host-check build and GPU engine).

Bit-exact for everything integer and for f64 (compared by bit pattern; NaN == NaN): counters,
estimator states, final clock, per-event (id, time, kind, pod, node, slot) logs, placements
(pod, node, assign_time) and per-pod start/finish/removal times.
"""
from __future__ import annotations

import math
import struct
from typing import Optional

import oracle_bridge as ob
from kubernetriks_amd.native import Capacities, RUN_UNTIL_ALL_FINISHED, RUN_UNTIL_TIME

ORACLE_STATUS = {0: "finished", 1: "time_limit", 2: "error", 3: "finished", 4: "running"}


def fbits(x: float) -> int:
    if isinstance(x, float) and math.isnan(x):
        return -1
    return struct.unpack("<q", struct.pack("<d", float(x)))[0]


def feq(a: float, b: float) -> bool:
    return fbits(a) == fbits(b)


GAUGE_ROWS = 1 << 14  # gauge recorder rows kept by run_pair's oracle and engine


def parity_caps(log: bool = True, fifo: int = 0, pruned: int = 0, gauges: int = 0) -> Capacities:
    c = Capacities()
    c.gauge_log = gauges
    c.delay_fifo = fifo
    c.pruned_scan = pruned
    c.event_log = (1 << 20) if log else 0
    c.placement_log = 1 << 20
    c.pod_records = 1
    # (the generated-name universes stay at their defaults: a replica that outgrows one is rerun in a
    # regrown batch by the engine itself, k10s.h k10s_engine_name_bounds)
    return c


def run_pair(engine_cls, scenario: str, mode: int = RUN_UNTIL_ALL_FINISHED, until: Optional[float] = None,
             max_time: float = 1e7, budget: int = 0, log: bool = True, params=None, fifo: int = 0,
             pruned: int = 0, ca_name_bound: int = 0, node_cache: int = 0):
    """Run the oracle and one engine replica on the same scenario; return (oracle dict, engine, res)."""
    o = ob.OracleSim(scenario, log=log, gauges=GAUGE_ROWS)
    if mode == RUN_UNTIL_ALL_FINISHED:
        st = o.run_until_all_finished(max_time)
    else:
        st = o.step_until_time(until)
    od = o.result(placements=True, log=log)
    od["status_name"] = ORACLE_STATUS[st] if not od["panicked"] else "error"
    caps = parity_caps(log, fifo, pruned, GAUGE_ROWS)
    caps.ca_name_bound = ca_name_bound
    caps.node_cache = node_cache
    eng = engine_cls(scenario, 1, params=params, caps=caps)
    if mode == RUN_UNTIL_ALL_FINISHED:
        eng.run_until_all_finished(max_time, budget)
    else:
        eng.step_until_time(until, budget)
    return od, eng


def compare(od: dict, eng, r: int = 0, log: bool = True, check_status: bool = True) -> list:
    """Return a list of human-readable mismatches (empty = bit-exact parity)."""
    er = eng.results()[r]
    bad = []
    if check_status:
        if od["panicked"] != (er["status"] == "error"):
            bad.append(f"panic mismatch: oracle={od['panicked']} ({od['panic']}) engine={er['status']} code={er['error_code']}")
        elif not od["panicked"] and od["status_name"] != er["status"]:
            bad.append(f"status: oracle={od['status_name']} engine={er['status']}")
    if not feq(od["time"], er["time"]):
        bad.append(f"clock: oracle={od['time']!r} engine={er['time']!r}")
    for k, v in od["counters"].items():
        if er["counters"][k] != v:
            bad.append(f"counter {k}: oracle={v} engine={er['counters'][k]}")
    for k, ov in od["estimators"].items():
        ev = er["estimators"][k]
        if ov[0] != ev[0] or not all(feq(a, b) for a, b in zip(ov[1:5], ev[1:5])) or list(ov[5]) != list(ev[5]):
            bad.append(f"estimator {k}: oracle={ov} engine={ev}")
    if od["unschedulable_len"] != er["unschedulable_len"]:
        bad.append(f"unschedulable_len: oracle={od['unschedulable_len']} engine={er['unschedulable_len']}")
    if od["active_len"] != er["active_len"]:
        bad.append(f"active_len: oracle={od['active_len']} engine={er['active_len']}")
    if od["node_counts"] != er["node_counts"]:
        bad.append(f"node_counts: oracle={od['node_counts']} engine={er['node_counts']}")
    # gauge recorder rows (when both sides recorded them)
    og = od.get("gauges") or []
    if og:
        eg = eng.gauges(r)
        if len(og) != len(eg):
            bad.append(f"gauges: oracle={len(og)} rows engine={len(eg)}")
        for i, (a, b) in enumerate(zip(og, eg)):
            if not all(feq(float(x), float(y)) for x, y in zip(a, b)):
                bad.append(f"gauge row #{i}: oracle={a} engine={b}")
                break
    # placements
    ep = eng.placements(r)
    op = [tuple(x) for x in od["placements"]]
    if len(ep) != len(op):
        bad.append(f"placements: oracle={len(op)} engine={len(ep)}")
    for i, (a, b) in enumerate(zip(op, ep)):
        if a[0] != b[0] or a[1] != b[1] or not feq(a[2], b[2]):
            bad.append(f"placement #{i}: oracle={a} engine={b}")
            break
    # pod records
    recs = eng.pod_records(r)
    for name, orec in od["pods"].items():
        state = {0: 1, 1: 2, 2: 3}[orec[5]]
        erec = recs.get(name)
        if erec is None:
            bad.append(f"pod {name}: missing in engine records")
            break
        if erec[3] != state or not feq(orec[2], erec[0]) or not feq(orec[3], erec[1]) or not feq(orec[4], erec[2]):
            bad.append(f"pod {name}: oracle={orec} engine={erec}")
            break
    if log:
        el = eng.event_log(r)
        ol = od["log"]
        if len(el) != len(ol):
            bad.append(f"event log length: oracle={len(ol)} engine={len(el)}")
        for i, (a, b) in enumerate(zip(ol, el)):
            # oracle: [id, time, kind, pod, node, slot]; engine: (seq, time, kind, pod, node, slot)
            if a[0] != b[0] or not feq(a[1], b[1]) or a[2] != b[2] or a[3] != b[3] or a[4] != b[4] or a[5] != b[5]:
                bad.append(f"event #{i}: oracle={a} engine={b}")
                break
    return bad
