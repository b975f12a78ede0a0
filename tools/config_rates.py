#!/usr/bin/env python3
"""Throughput of the BASELINE configs besides C3 (tooling; SURVEY.md §8(d) "aggregate placements/s,
attempts/s and events/s at C2, C3 and C4"): the GPU engine batch and the CPU baseline side by side.

  c2   1,024 replicas of the 31-node default cluster (src/config.yaml:45-68), replica r running the
       first ceil(U_r * 10,000) pods of a test_determinism-style trace (workloads.c2_survey_parts),
       seed-perturbed, run until all pods finished
  c4   1,024 replicas of the C4 scenario (test_hpa.rs pod group + config.yaml:14-33 CA groups + a
       400-pod burst, workloads.c4_parts), seed-perturbed, stepped to t = 3,000 s (step_until_time:
       the pod group never finishes)

GPU: one engine batch per config, wall time of k10s_engine_run (HIP events) and of the call.
CPU: the repo's oracle (kind "port": a C++ restatement of the reference; the Rust reference cannot
be built in this image), one process per usable host core, each simulating one replica of the same
config (its own seed / trace length) for at most --cpu-seconds of wall time; rates are the sum over
processes of (work done / wall time).  Prints one JSON object.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def _config(name):
    from kubernetriks_amd import workloads as wl
    if name == "c2":
        parts = wl.c2_survey_parts()
        return parts, (lambda d, n: wl.c2_survey_params(d, n)), None
    if name == "c4":
        parts = wl.c4_parts(n_batch_pods=400, seed=7)
        return parts, (lambda d, n: wl.replica_params(d, n, base_seed=7, perturb=True)), 3000.0
    raise SystemExit(f"unknown config {name}")


def _cpu_job(args):
    scn, until, cap = args
    import oracle_bridge as ob
    o = ob.OracleSim(scn)
    t0 = time.perf_counter()
    t_sim, done = 0.0, False
    while time.perf_counter() - t0 < cap:
        t_sim += 50.0
        if until is not None and t_sim >= until:
            o.step_until_time(until)
            done = True
            break
        o.step_until_time(t_sim)
        r = o.result()
        if r["panicked"]:
            done = True
            break
        if until is None and r["counters"]["terminated_pods"] >= r["counters"]["total_pods_in_trace"]:
            o.run_until_all_finished(1e7)
            done = True
            break
    wall = time.perf_counter() - t0
    c = o.result()["counters"]
    return c["placements"], c["attempts"], c["events"], wall, done


def cpu_rates(name, cpu_seconds):
    from multiprocessing import get_context
    import bench
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.native import ReplicaParams
    from hostcheck_bridge import HostEngine
    from kubernetriks_amd.scenario import scenario_text
    (cfg, cluster, workload), pfn, until = _config(name)
    usable, info = bench.host_cores()
    scn = scenario_text(cfg, cluster, workload)
    params = pfn(HostEngine(scn, 1).default_params(), usable)
    jobs = [(wl.replica_scenario(cfg, cluster, workload, p), until, cpu_seconds) for p in params]
    with get_context("spawn").Pool(usable) as pool:
        res = pool.map(_cpu_job, jobs)
    return {"placements_per_s": sum(r[0] / r[3] for r in res), "attempts_per_s": sum(r[1] / r[3] for r in res),
            "events_per_s": sum(r[2] / r[3] for r in res), "cores": usable, "host": info, "kind": "port",
            "replicas_completed": sum(1 for r in res if r[4]), "wall_cap_s": cpu_seconds,
            "sample": f"{usable} processes x 1 replica of {name} each (own seed / trace length), up to "
                      f"{cpu_seconds:.0f} s of wall time each"}


def gpu_rates(name, R):
    import numpy as np
    from kubernetriks_amd.build import build
    build()
    from kubernetriks_amd.native import Engine, version
    from kubernetriks_amd.scenario import scenario_bulk
    (cfg, cluster, workload), pfn, until = _config(name)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    params = pfn(Engine(scn, 1, pods_blob=blob).default_params(), R)
    eng = Engine(scn, R, params=params, pods_blob=blob)
    out = {}
    for rep in range(2):   # first run includes one-time costs; report the second
        eng.reset()
        t0 = time.perf_counter()
        ms = eng.step_until_time(until) if until is not None else eng.run_until_all_finished(1e7)
        wall = time.perf_counter() - t0
        c = eng.counter_matrix().sum(axis=0, dtype=np.uint64).astype(np.int64)
        st = {}
        for r in eng.raw_results():
            st[int(r.status)] = st.get(int(r.status), 0) + 1
        out = {"replicas": R, "kernel_ms": ms, "wall_s": wall, "placements": int(c[12]), "attempts": int(c[13]),
               "events": int(c[14]), "placements_per_s": int(c[12]) / wall, "attempts_per_s": int(c[13]) / wall,
               "events_per_s": int(c[14]) / wall, "replica_status": st, "engine": version()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c4")
    ap.add_argument("--replicas", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    out = {}
    for name in a.configs.split(","):
        row = {}
        if not a.no_gpu:
            row["gpu"] = gpu_rates(name, a.replicas)
            print(f"[{name}] gpu {row['gpu']['placements_per_s']:.4g} placements/s", file=sys.stderr, flush=True)
        if not a.no_cpu:
            row["cpu_baseline"] = cpu_rates(name, a.cpu_seconds)
            print(f"[{name}] cpu {row['cpu_baseline']['placements_per_s']:.4g} placements/s", file=sys.stderr, flush=True)
        out[name] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
