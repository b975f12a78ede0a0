#!/usr/bin/env python3
"""Finish-time spread of one k10s_run_kernel launch (tooling; needs a K10S_WALL=1 variant build,
loaded with K10S_LIB=build/libk10s_WALL1.so).

Each replica records the 100 MHz realtime counter at its start and end and its hardware ids
(HW_ID: wave/SIMD/CU/SE, XCC_ID) in its profile slots.  Prints one JSON object: the distribution
of per-replica wall times and finish times over the launch, the time-weighted number of live
replicas per SIMD, and the per-replica event counts, so the tail of the resident round can be
told apart from per-replica work differences.
usage: python tools/wall_spread.py [--workload c3|c3_backlog] [--replicas R]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def pct(a, qs=(0, 1, 5, 25, 50, 75, 95, 99, 100)):
    import numpy as np
    return {str(q): float(np.percentile(a, q)) for q in qs}


def main():
    import numpy as np
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3")
    ap.add_argument("--replicas", type=int, default=8192)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--pods", type=int, default=16384)
    ap.add_argument("--arrival-window", type=float, default=1200.0)
    a = ap.parse_args()
    import bench
    from kubernetriks_amd import ensemble
    from kubernetriks_amd.native import Capacities, Engine
    from kubernetriks_amd.scenario import scenario_bulk
    cfg, cluster, workload, desc, sweep = bench.build_workload(a)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    probe = Engine(scn, 1, pods_blob=blob)
    params = ensemble.shard_params(probe.default_params(), a.replicas, 0, base_seed=123, perturb=True, sweep=sweep)
    del probe
    eng = Engine(scn, a.replicas, params=params, caps=Capacities(), pods_blob=blob)
    eng.run_until_all_finished(max_time=1e7)      # warm-up launch
    eng.reset()
    ms = eng.run_until_all_finished(max_time=1e7)
    prof = eng.profile()
    t0 = np.array([p["loop"] for p in prof], dtype=np.float64)
    t1 = np.array([p["select"] for p in prof], dtype=np.float64)
    hw = np.array([p["consume"] for p in prof], dtype=np.uint64)
    xcc = np.array([p["dispatch"] for p in prof], dtype=np.uint64)
    ev = eng.counter_matrix()[:, 14].astype(np.float64)
    base = t0.min()
    start = (t0 - base) / 1e5          # ms (100 MHz)
    end = (t1 - base) / 1e5
    dur = end - start
    span = end.max()
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 3
    key = ((xcc * 4 + se) * 2 + sh) * 64 + cu * 4 + simd
    _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    simd_end = np.zeros(cnt.size)
    np.maximum.at(simd_end, inv, end)
    simd_sum = np.zeros(cnt.size)
    np.add.at(simd_sum, inv, dur)
    out = {
        "workload": desc, "kernel_ms_hip_event": ms, "span_ms": span,
        "start_ms": pct(start), "end_ms": pct(end), "duration_ms": pct(dur),
        "events_per_replica": pct(ev),
        "corr_duration_events": float(np.corrcoef(dur, ev)[0, 1]),
        "ns_per_event": pct(dur * 1e6 / np.maximum(ev, 1)),
        "mean_live_replicas_per_simd": float(dur.sum() / (cnt.size * span)),
        "simds": int(cnt.size), "replicas_per_simd": pct(cnt),
        "simd_last_end_ms": pct(simd_end),
        "simd_busy_fraction": pct(simd_sum / (cnt * span)),
        "by_xcc_mean_duration_ms": {int(x): float(dur[xcc == x].mean()) for x in np.unique(xcc)},
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
