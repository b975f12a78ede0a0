#!/usr/bin/env python3
"""Run a bench workload slice through one engine library (K10S_LIB selects a variant build) in budgeted
launches and print one JSON object: per replica the status, error code, clock bits and counters
(tooling; tests/test_variants.py compares a variant build's rows with the product build's).

Usage: [K10S_LIB=build/libk10s_<variant>.so] tools/variant_run.py WORKLOAD REPLICAS NODES PODS BUDGET"""
import argparse
import json
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import bench
    from kubernetriks_amd import ensemble
    from kubernetriks_amd.native import Engine, RUN_UNTIL_ALL_FINISHED, version
    from kubernetriks_amd.scenario import scenario_bulk
    wl, R, nodes, pods, budget = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    a = argparse.Namespace(workload=wl, nodes=nodes, pods=pods, arrival_window=1200.0, replicas=R,
                           score_plugins="least")
    cfg, cluster, workload, desc, sweep = bench.build_workload(a)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    defaults = Engine(scn, 1, pods_blob=blob).default_params()
    params = ensemble.shard_params(defaults, R, 0, base_seed=123, perturb=True, sweep=sweep)
    eng = Engine(scn, R, params=params, pods_blob=blob)
    launches = 0
    while True:
        eng.step_async(RUN_UNTIL_ALL_FINISHED, 0.0, 1e7, budget)
        eng.sync()
        launches += 1
        if all(r.status != 0 for r in eng.raw_results()) or launches > 100000:
            break
    rows = []
    for r in eng.raw_results():
        rows.append({"status": int(r.status), "error_code": int(r.error_code), "error_kind": int(r.error_kind),
                     "clock_bits": struct.unpack("<Q", struct.pack("<d", r.clock))[0],
                     "counters": [int(x) for x in r.counters]})
    print(json.dumps({"engine": version(), "lib": os.environ.get("K10S_LIB", "build/libk10s.so"),
                      "launches": launches, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
