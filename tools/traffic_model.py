#!/usr/bin/env python3
"""Memory-touch model of the run kernel per event kind and HBM section (tooling; VERDICT r04 #5's
attribution).  Builds the TEST-ONLY host engine (tests/hostcheck) with clang's load/store tracing
(-fsanitize-coverage=trace-loads,trace-stores) and -DK10S_TRAFFIC_MODEL, runs one replica of a bench
workload, and reports per event kind: dispatches, the distinct 128-B lines read and 64-B chunks
written per dispatch in each section of the replica's HBM region (header excluded: LDS on the
device), "cold" (nothing survives between events) and "warm" reads (a per-replica LRU of
--lru lines, the replica's share of L2).  Events handled inside a run, a window or a fused relay
count under the dispatch that entered them.
Usage: tools/traffic_model.py [c3|c3_backlog] [nodes] [pods] [--lru N] > profiles/<round>_traffic_model_<wl>.json"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def build(out):
    tm = os.path.join(REPO, "tools", "traffic_model")
    hc = os.path.join(REPO, "tests", "hostcheck")
    inc = ["-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "kubernetriks_amd", "csrc")]
    objs = []
    for src, flags in [(os.path.join(tm, "traffic_rt.cpp"), []),
                       (os.path.join(REPO, "kubernetriks_amd", "csrc", "k10s_builder.cpp"), []),
                       (os.path.join(hc, "hostcheck.cpp"),
                        ["-DK10S_TRAFFIC_MODEL", "-fsanitize-coverage=inline-8bit-counters,trace-loads,trace-stores"])]:
        o = os.path.join(REPO, "build", "tm_" + os.path.basename(src) + ".o")
        subprocess.check_call([CLANG, "-O1", "-std=c++17", "-fPIC", "-ffp-contract=off", "-w", *inc, *flags, "-c", src, "-o", o])
        objs.append(o)
    subprocess.check_call([CLANG, "-shared", "-o", out, *objs])
    for o in objs:
        os.unlink(o)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lru = 32
    if "--lru" in sys.argv:
        lru = int(sys.argv[sys.argv.index("--lru") + 1])
        args = [a for a in args if a != str(lru)]
    wl_name = args[0] if args else "c3"
    nodes = int(args[1]) if len(args) > 1 else 4096
    pods = int(args[2]) if len(args) > 2 else 8192
    out = os.path.join(REPO, "build", "libk10s_traffic_model.so")
    build(out)
    os.environ["K10S_HOSTCHECK_LIB"] = out
    import hostcheck_bridge as hb
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.native import EVENT_KIND_NAMES
    from kubernetriks_amd.scenario import SimulationConfig, scenario_text
    window = 1200.0 * pods / 16384
    if wl_name == "c3_backlog":
        cluster, workload = wl.c3_backlog_traces(nodes, pods, window)
    else:
        cluster, workload = wl.c3_traces(n_nodes=nodes, n_pods=pods, arrival_window=window, seed=123)
    L = hb.lib()
    L.k10s_tm_lru(lru)
    eng = hb.HostEngine(scenario_text(SimulationConfig(), cluster, workload), 1)
    eng.run_until_all_finished(max_time=1e7)
    path = os.path.join(REPO, "build", "traffic_model.json")
    assert L.k10s_tm_dump(path.encode()) == 0
    raw = json.load(open(path))
    counters = eng.results()[0]["counters"]
    events = counters["events"]
    kinds, tot = {}, {"cold_rd_B": 0.0, "cold_wr_B": 0.0, "warm_rd_B": 0.0}
    by_sec = {}
    for k, v in raw["kinds"].items():
        name = EVENT_KIND_NAMES.get(int(k), k)
        d = v["dispatches"]
        row = {"dispatches": int(d)}
        for key, unit in (("cold_rd_lines", 128), ("cold_wr_chunks", 64), ("warm_rd_lines", 128)):
            secs = v[key]
            row[key.replace("lines", "B").replace("chunks", "B") + "_per_dispatch"] = {s: round(n * unit / d, 1) for s, n in secs.items()}
            b = sum(secs.values()) * unit
            tot[key.split("_")[0] + "_" + key.split("_")[1] + "_B"] += b
            for s, n in secs.items():
                by_sec.setdefault(key, {}).setdefault(s, 0.0)
                by_sec[key][s] += n * unit
        kinds[name] = row
    print(json.dumps({"workload": wl_name, "nodes": nodes, "pods": pods, "lru_lines": lru, "events": events,
                      "section_offsets": raw["sections"], "stride": raw["stride"],
                      "counters": {k: counters[k] for k in ("placements", "attempts", "nodes_read")},
                      "per_event_B": {k: round(v / events, 1) for k, v in tot.items()},
                      "per_event_B_by_section": {k: {s: round(v / events, 1) for s, v in sorted(d.items(), key=lambda x: -x[1])}
                                                 for k, d in by_sec.items()},
                      "kinds": kinds}, indent=1))


if __name__ == "__main__":
    main()
