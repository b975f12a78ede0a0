#!/usr/bin/env python3
"""Run a bench workload slice through a sanitizer build of the host engine (tooling for the round-3
K10S_PROF hang, VERDICT r03 "What's weak" 2): the same engine code with -fsanitize=address,undefined
and the given -D knobs (default K10S_PROF=1, the header layout the profile build implies), in
budgeted "launches" like tools/launch_trace.py, one progress line per launch.  An out-of-bounds
access into a RepHdr array or a replica section aborts with the sanitizer's report.

Usage: tools/hang_hostcheck.py [--workload c5_autoscaled] [--replicas 64] [--budget 1000000]
                               [--launches 40] [--define K10S_PROF=1 ...]
The process re-executes itself once with the sanitizer runtime preloaded (before anything touches
a GPU: this is a host-only tool)."""
import argparse
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def build_lib(defines):
    tag = "_".join(d.replace("K10S_", "").replace("=", "") for d in defines) or "plain"
    out = os.path.join(REPO, "build", f"libk10s_hostcheck_san_{tag}.so")
    flags = ("-O1 -g -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function "
             "-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer "
             + " ".join(f"-D{d}" for d in defines))
    subprocess.check_call(["make", "-s", "-B", "-C", os.path.join(REPO, "tests", "hostcheck"),
                           f"OUT={out}", f"CXXFLAGS={flags}"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5_autoscaled")
    ap.add_argument("--replicas", type=int, default=64)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--pods", type=int, default=16384)
    ap.add_argument("--budget", type=int, default=1000000)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--define", action="append", default=None)
    a = ap.parse_args()
    defines = a.define if a.define is not None else ["K10S_PROF=1"]
    if not os.environ.get("K10S_HANG_CHILD"):
        lib = build_lib(defines)
        asan = subprocess.check_output(["gcc", "-print-file-name=libasan.so"], text=True).strip()
        ubsan = subprocess.check_output(["gcc", "-print-file-name=libubsan.so"], text=True).strip()
        env = dict(os.environ, K10S_HANG_CHILD="1", K10S_HOSTCHECK_LIB=lib, LD_PRELOAD=f"{asan}:{ubsan}",
                   ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
        sys.exit(subprocess.call([sys.executable] + sys.argv, env=env))

    import bench
    from hostcheck_bridge import HostEngine
    from kubernetriks_amd import ensemble
    from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED
    from kubernetriks_amd.scenario import scenario_bulk
    ns = argparse.Namespace(workload=a.workload, nodes=a.nodes, pods=a.pods, arrival_window=1200.0,
                            replicas=a.replicas, score_plugins="least")
    cfg, cluster, workload, desc, sweep = bench.build_workload(ns)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    probe = HostEngine(scn, 1, pods_blob=blob)
    defaults = probe.default_params()
    del probe
    params = ensemble.shard_params(defaults, a.replicas, 0, base_seed=123, perturb=True, sweep=sweep)
    eng = HostEngine(scn, a.replicas, params=params, pods_blob=blob)
    t0 = time.time()
    for i in range(a.launches):
        eng.run(RUN_UNTIL_ALL_FINISHED, 0.0, 1e7, a.budget)
        res = eng.raw_results()
        running = [r for r in res if r.status == 0]
        ev = int(eng.counter_matrix().sum(axis=0)[14])
        clk = min((r.clock for r in running), default=None)
        print(f"launch {i}: running {len(running)} events {ev} min_clock {clk} t={time.time() - t0:.1f}s", flush=True)
        if not running:
            break
    st = {}
    for r in eng.raw_results():
        st[r.status] = st.get(r.status, 0) + 1
    print("status counts", st, "events", int(eng.counter_matrix().sum(axis=0)[14]), flush=True)


if __name__ == "__main__":
    main()
