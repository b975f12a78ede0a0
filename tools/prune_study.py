#!/usr/bin/env python3
"""Block-pruning study on the host engine (tooling, not product): builds the test-only host engine
with -DK10S_PRUNE_STUDY, runs one replica of a bench workload and prints, for block sizes 16..512,
how many node-cache entries an exact block-pruned scan (tight componentwise block maxima, best-first
block order, strict skip; k10s_engine.h k10s_prune_study) would read per scan, against the full
scan's N.
Usage: tools/prune_study.py [c3|c3_backlog] [nodes] [pods]"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    wl_name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    pods = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    out = os.path.join(REPO, "build", "libk10s_prunestudy.so")
    defs = os.path.join(REPO, "build", "prunestudy_defs.cpp")
    with open(defs, "w") as f:
        f.write('#include <cstdint>\nextern "C" uint64_t k10s_prune_stats[48];\nuint64_t k10s_prune_stats[48];\n')
    hc = os.path.join(REPO, "tests", "hostcheck")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DK10S_PRUNE_STUDY", "-DK10S_TILE_PRUNE=0", "-DK10S_FRONT=0", "-shared",
                           "-o", out, os.path.join(hc, "hostcheck.cpp"),
                           os.path.join(REPO, "kubernetriks_amd", "csrc", "k10s_builder.cpp"), defs])
    import hostcheck_bridge as hb
    hb.LIB_PATH = out
    hb.build = lambda: None
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.scenario import SimulationConfig, scenario_text
    if wl_name == "c3_backlog":
        cluster, workload = wl.c3_backlog_traces(nodes, pods, 1200.0)
    else:
        cluster, workload = wl.c3_traces(n_nodes=nodes, n_pods=pods, arrival_window=1200.0, seed=123)
    eng = hb.HostEngine(scenario_text(SimulationConfig(), cluster, workload), 1)
    eng.run_until_all_finished(max_time=1e7)
    st = (ctypes.c_uint64 * 48).in_dll(hb.lib(), "k10s_prune_stats")
    scans = max(int(st[12]), 1)
    rows = {}
    for i in range(6):
        B = 16 << i
        rows[B] = {"entries_per_scan": round(st[2 * i] / scans, 1), "blocks_per_scan": round(st[2 * i + 1] / scans, 2),
                   "frac_of_full": round(st[2 * i] / scans / nodes, 4)}
    att = max(int(st[14]), 1)
    depth = {str(d) + ("+" if d == 15 else ""): round(st[16 + d] / att, 4) for d in range(1, 16)}
    print(json.dumps({"workload": wl_name, "nodes": nodes, "pods": pods, "scans": scans, "by_block": rows,
                      "cycles": int(st[13]), "attempts_per_cycle": round(att / max(int(st[13]), 1), 2),
                      "distinct_reserved_per_cycle": round(st[15] / max(int(st[13]), 1), 2),
                      "snapshot_depth_share": depth,
                      "per_scan_nodes_tied": round(st[40] / scans, 1), "within_1e-5": round(st[41] / scans, 1),
                      "within_1e-4": round(st[42] / scans, 1), "within_1e-3": round(st[43] / scans, 1),
                      "pareto_front_per_scan": round(st[44] / scans, 1),
                      "block64_front_mean": round(st[45] / scans / ((nodes + 63) // 64), 2),
                      "block64_fronts_over_8_per_scan": round(st[46] / scans, 3), "block64_front_max": int(st[47])}, indent=1))


if __name__ == "__main__":
    main()
