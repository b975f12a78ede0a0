#!/usr/bin/env python3
"""Budgeted launches of a bench workload with one progress line per launch (tooling: diagnoses a
replica that stops finishing).  Usage: tools/launch_trace.py WORKLOAD REPLICAS BUDGET MAX_LAUNCHES
(K10S_LIB selects a variant build).  Prints per launch: replicas still running, total events,
minimum clock of the running replicas."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    from kubernetriks_amd import ensemble
    from kubernetriks_amd.native import Engine, RUN_UNTIL_ALL_FINISHED
    from kubernetriks_amd.scenario import scenario_bulk
    wl, R, budget, nmax = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    a = argparse.Namespace(workload=wl, nodes=4096, pods=16384, arrival_window=1200.0, replicas=R, score_plugins="least")
    cfg, cluster, workload, desc, sweep = bench.build_workload(a)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    probe = Engine(scn, 1, pods_blob=blob)
    defaults = probe.default_params()
    del probe
    params = ensemble.shard_params(defaults, R, 0, base_seed=123, perturb=True, sweep=sweep)
    eng = Engine(scn, R, params=params, pods_blob=blob)
    t0 = time.time()
    for i in range(nmax):
        eng.step_async(RUN_UNTIL_ALL_FINISHED, 0.0, 1e7, budget)
        eng.sync()
        res = eng.raw_results()
        running = [r for r in res if r.status == 0]
        ev = int(eng.counter_matrix().sum(axis=0)[14])
        clk = min((r.clock for r in running), default=None)
        errs = {}
        for r in res:
            if r.status == 2:
                k = (r.error_code, r.error_kind)
                errs[k] = errs.get(k, 0) + 1
        print(f"launch {i}: running {len(running)} events {ev} min_clock {clk} errors(code,kind) {errs} "
              f"t={time.time() - t0:.1f}s", flush=True)
        if not running:
            break
    st = {}
    for r in eng.raw_results():
        st[r.status] = st.get(r.status, 0) + 1
    print("status counts", st, "events", int(eng.counter_matrix().sum(axis=0)[14]), flush=True)


if __name__ == "__main__":
    main()
