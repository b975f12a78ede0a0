#!/usr/bin/env python3
"""Benchmark: pod placements/sec of the MI355X batched-ensemble engine on 4k-node clusters.

Workload (BASELINE.json configs[2] shape, the metric's "4k-node clusters"): C3 — every GPU runs
R replicas (default 8,192) of a 4,096-node Alibaba-like cluster, each replica a seed-perturbed copy
of one synthetic 16,384-pod Alibaba-like trace (integer arrival seconds); a step simulates every
replica from initialize() until RunUntilAllPodsAreFinished stops it.  Replicas are sharded over
ranks with distinct seeds (weak scaling: R per GPU); the only collective is one RCCL all-reduce of
the counter vector per measurement (the reference has no data-path exchange).

Prints ONE JSON line (rank 0).  `value` = placements of all ranks / max-over-ranks wall time of
the timed steps.  `roofline`: the dominant kernel is k10s_run_kernel (the whole event loop incl. the
scheduling scans); algorithmic bytes per launch = Σ_attempts (12·|node cache| + 12) + 12·placements
(SURVEY.md §8(d)), divided by the launch's HIP-event time, against the 8 TB/s HBM3E peak.
`cpu_baseline`: the repo's CPU oracle (a string-keyed restatement of the reference, kind "port";
the Rust reference cannot be built here) on a bounded sample of the same workload, one process
per core.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12  # MI355X HBM3E peak, MI355X_MICROARCH.md "Chip-level parameters"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--replicas", type=int, default=8192, help="replicas per GPU")
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--pods", type=int, default=16384)
    ap.add_argument("--arrival-window", type=float, default=1200.0)
    ap.add_argument("--budget", type=int, default=0, help="max events per replica per launch (0 = one launch)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = min(16, cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-scan-kernel", action="store_true", help="skip the scheduling-kernel-alone measurement")
    ap.add_argument("--pruned-scan", action="store_true", help="exact block-bound pruned scan (DESIGN.md §3)")
    ap.add_argument("--profile", action="store_true", help="print the K10S_PROF cycle attribution (variant builds)")
    return ap.parse_args()


def cpu_worker(args_tuple):
    """One core: the oracle on one replica's materialized trace for ~`seconds` of wall time."""
    scn, seconds = args_tuple
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bridge as ob
    o = ob.OracleSim(scn)
    t0 = time.perf_counter()
    t_sim = 0.0
    while time.perf_counter() - t0 < seconds:
        t_sim += 20.0
        o.step_until_time(t_sim)
        r = o.result()
        if r["panicked"] or t_sim > 1e6:
            break
        if r["counters"]["terminated_pods"] >= r["counters"]["total_pods_in_trace"]:
            break
    wall = time.perf_counter() - t0
    c = o.result()["counters"]
    return c["placements"], c["attempts"], c["events"], wall, t_sim


def cpu_baseline(args, cfg, cluster, workload, params):
    from multiprocessing import get_context
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.scenario import scenario_text
    workers = args.cpu_workers or min(16, os.cpu_count() or 1)
    jobs = [(scenario_text(cfg, cluster, wl.perturb_workload(workload, params[i].seed)), args.cpu_seconds)
            for i in range(workers)]
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bridge as ob
    ob.build_oracle()
    with get_context("fork").Pool(workers) as pool:
        res = pool.map(cpu_worker, jobs)
    rate = sum(p / w for p, _, _, w, _ in res)
    sample = (f"{workers} processes x 1 replica of the same C3 workload ({args.nodes} nodes, {args.pods} pods, "
              f"seed-perturbed), each run ~{args.cpu_seconds:.0f}s of wall time from t=0; "
              f"{sum(r[0] for r in res)} placements, {sum(r[2] for r in res)} events in total")
    return {"value": rate, "unit": "placements/s", "cores": workers, "kind": "port", "sample": sample,
            "per_core_placements_per_s": rate / workers,
            "attempts_per_s": sum(a / w for _, a, _, w, _ in res),
            "events_per_s": sum(e / w for _, _, e, w, _ in res)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    torch.cuda.set_device(local_rank)

    from kubernetriks_amd.build import build
    build()
    from kubernetriks_amd import ensemble
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.native import NUM_COUNTERS, Capacities, Engine, version
    from kubernetriks_amd.scenario import SimulationConfig, scenario_bulk

    cfg = SimulationConfig()
    cluster, workload = wl.c3_traces(args.nodes, args.pods, args.arrival_window)
    # cluster trace as text, the 16k create_pod events as the binary block (k10s_engine_create_bulk)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    R = args.replicas
    probe = Engine(scn, 1, device=local_rank, pods_blob=blob)
    defaults = probe.default_params()
    probe.close()
    params = ensemble.shard_params(defaults, R, rank, base_seed=123, perturb=True)  # replicas [rank*R, (rank+1)*R)
    t = time.perf_counter()
    caps = Capacities()
    caps.pruned_scan = 1 if args.pruned_scan else 0
    eng = Engine(scn, R, params=params, caps=caps, device=local_rank, pods_blob=blob)
    log(f"[rank {rank}] engine: {R} replicas x {eng.replica_bytes / 2**20:.1f} MiB, init {time.perf_counter() - t:.2f}s")

    def one_step():
        eng.reset()
        return eng.run_until_all_finished(max_time=1e7, max_events_per_launch=args.budget)

    for i in range(args.warmup):
        t = time.perf_counter()
        one_step()
        log(f"[rank {rank}] warmup {i}: {time.perf_counter() - t:.2f}s")

    import numpy as np
    counters = np.zeros(NUM_COUNTERS, dtype=np.float64)
    kernel_ms = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ms = one_step()
        kernel_ms.append(ms)
        res = eng.raw_results()
        for r in res:
            for k in range(NUM_COUNTERS):
                counters[k] += r.counters[k]
        log(f"[rank {rank}] step {i}: run {ms:.1f} ms")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    statuses, errors = {}, {}
    for r in eng.raw_results():
        statuses[r.status] = statuses.get(r.status, 0) + 1
        if r.status == 2:
            key = f"{r.error_code}@kind{r.error_kind}"
            errors[key] = errors.get(key, 0) + 1
    if statuses.get(2):
        log(f"[rank {rank}] WARNING: {statuses[2]} replicas ended in error: {errors}")

    # cross-rank reduction (RCCL over xGMI): max of the timings, sum of the counters; the per-replica
    # estimators of the last step are gathered in rank order into the job's ensemble summary
    elapsed, mean_kernel_ms = ensemble.max_over_ranks([elapsed, sum(kernel_ms) / len(kernel_ms)])
    c = ensemble.sum_over_ranks(counters.tolist())
    summary = ensemble.ensemble_summary(eng.raw_results()).as_dict()
    placements, attempts, events, scanned, nread = c[12], c[13], c[14], c[15], c[16]
    value = placements / elapsed

    # roofline for the dominant kernel (per launch, this rank's launch time, all-rank bytes / world)
    per_launch_bytes = (12.0 * scanned + 12.0 * attempts + 12.0 * placements) / (args.steps * world)
    achieved = per_launch_bytes / (mean_kernel_ms * 1e-3)
    # what the scans actually read (pruned scan: block bounds + scanned blocks + bound upkeep)
    touched_bytes = (12.0 * nread + 12.0 * attempts + 12.0 * placements) / (args.steps * world)
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", "pmc_run_kernel.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            # only a PMC pass over this exact kernel build, config and scan mode counts
            if pm.get("config") == [R, args.nodes, args.pods] and pm.get("engine") == version() and \
                    pm.get("scan_mode") == ("pruned" if args.pruned_scan else "full"):
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "pod placements/sec (whole node, 1/2/4/8 GPUs) at 4k-node clusters; % HBM roofline",
        "value": value,
        "unit": "placements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: Alibaba-like 4096-node clusters and 16384-pod traces (notebook statistics), seed-perturbed per replica",
        "config": {"workload": f"C3: {R} replicas/GPU x {args.nodes}-node Alibaba-like cluster, {args.pods} pods/replica, "
                               "run until all pods finished (RunUntilAllPodsAreFinished)",
                   "replicas_per_gpu": R, "total_replicas": R * world, "nodes": args.nodes, "pods_per_replica": args.pods,
                   "parallelism": f"replica-sharded x{world} (RCCL all-reduce of counters and histograms only)"},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK, "traffic": traffic,
                     "kernel": "k10s_run_kernel", "kernel_ms_per_launch": mean_kernel_ms,
                     "algorithmic_bytes_per_launch": per_launch_bytes,
                     "scan_mode": "pruned" if args.pruned_scan else "full",
                     "touched_bytes_per_launch": touched_bytes,
                     "touched_GBps": touched_bytes / (mean_kernel_ms * 1e-3) / 1e9},
        "engine": version(),
        "rates": {"placements_per_s": value, "attempts_per_s": attempts / elapsed, "events_per_s": events / elapsed},
        "totals": {"placements": placements, "attempts": attempts, "events": events, "nodes_scanned": scanned,
                   "nodes_read": nread,
                   "replica_status": {str(k): v for k, v in statuses.items()}, "replica_errors": errors},
        "ensemble": {"replicas": summary["replicas"], "replica_status": summary["replica_status"],
                     "counters": {k: summary["counters"][k] for k in ("total_pods_in_trace", "pods_succeeded",
                                                                       "terminated_pods", "placements", "events")},
                     "timings": summary["timings"], "histograms": summary.get("histograms")},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args, cfg, cluster, workload, params)
        except Exception as ex:  # the GPU number stands on its own
            log("cpu baseline failed:", ex)
            out["cpu_baseline"] = None
    if rank == 0 and not args.no_scan_kernel:
        # the scheduling-cycle kernel alone (k10s_schedule_one_batch over C3-sized node caches in HBM)
        try:
            from kubernetriks_amd.scanbench import measure
            out["scheduling_kernel"] = measure(R, args.nodes)
        except Exception as ex:
            log("scan kernel measurement failed:", ex)
            out["scheduling_kernel"] = None
    if args.profile:
        prof = eng.profile()
        tot = {k: float(sum(p[k] for p in prof)) for k in prof[0]}
        loop = tot["loop"] or 1.0
        out["profile"] = {"cycles_total": tot, "share_of_loop": {k: v / loop for k, v in tot.items() if k != "scans"},
                          "cycles_per_event": loop / max(events / args.steps / world, 1.0),
                          "scan_cycles_per_scan": tot["scan"] / max(tot["scans"], 1.0)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
