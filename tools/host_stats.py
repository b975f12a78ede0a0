#!/usr/bin/env python3
"""Event-path statistics of the engine logic on the host (tooling, not product): builds the
test-only host engine (tests/hostcheck) with -DK10S_HOST_STATS into build/libk10s_hoststats.so, runs
one replica of a bench workload to completion and prints, per delivered event, how often each path of
the event queue was taken (FIFO pops, window refills from the HBM ring, heap pops, source-list fast
path vs full update, emissions into a window / the HBM ring / the heap).
Usage: tools/host_stats.py [c3|c3_backlog] [nodes] [pods]"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
NAMES = ["events", "fifo_pop", "refill", "heap_pop", "trace_pop", "sl_fast", "sl_update", "emit_window",
         "emit_ring", "emit_heap", "sl_dirty", "scans"]


def main():
    wl_name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    pods = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    out = os.path.join(REPO, "build", "libk10s_hoststats.so")
    defs = os.path.join(REPO, "build", "hoststats_defs.cpp")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(defs, "w") as f:
        f.write('#include <cstdint>\nextern "C" uint64_t k10s_host_stats[48];\nuint64_t k10s_host_stats[48];\n')
    hc = os.path.join(REPO, "tests", "hostcheck")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DK10S_HOST_STATS", "-shared",
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
    st = (ctypes.c_uint64 * 48).in_dll(hb.lib(), "k10s_host_stats")
    v = {n: int(st[i]) for i, n in enumerate(NAMES)}
    ev = max(v["events"], 1)
    rings = ["as_to_ps", "ps_to_sched", "sched_to_as", "assign", "as_to_node", "as_to_ca", "as_to_hpa", "now"]
    per_ring = {r: {"pops": int(st[20 + i]), "refills": int(st[12 + i])} for i, r in enumerate(rings)}
    print(json.dumps({"workload": wl_name, "nodes": nodes, "pods": pods, "counts": v,
                      "per_event": {n: round(v[n] / ev, 4) for n in NAMES if n != "events"},
                      "refills_per_fifo_pop": round(v["refill"] / max(v["fifo_pop"], 1), 4),
                      "rings": per_ring, "aq_pops": int(st[29]), "aq_hbm_reads": int(st[28]),
                      "sl_insert_pos_0_1_2_3plus": [int(st[32 + i]) for i in range(4)],
                      "runs": int(st[38]), "run_events": int(st[39]), "runs_refused": int(st[40]),
                      "windows": int(st[41]), "window_events": int(st[42]),
                      "tile_picks": int(st[43]), "tile_picks_with_rescan": int(st[44]), "fused_finish_relays": int(st[45]),
                      "next_event_emitted_by_previous": round(int(st[36]) / ev, 4),
                      "next_event_emitted_by_previous_fifo": round(int(st[37]) / ev, 4)}, indent=1))


if __name__ == "__main__":
    main()
