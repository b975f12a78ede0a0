#!/usr/bin/env python3
"""Benchmark: pod placements/sec of the MI355X batched-ensemble engine on 4k-node clusters.

Workloads (BASELINE.json configs[2] and [4] shapes, the metric's "4k-node clusters"):
  c3             every GPU runs R replicas (default 8,192) of a 4,096-node Alibaba-like cluster, each
                 a seed-perturbed copy of one synthetic 16,384-pod Alibaba-like trace (integer arrival
                 seconds, notebook statistics); light load (rho ~ 0.007 of the RAM-bound capacity:
                 ~2,600 concurrent pods on room for ~360 k), every attempt places its pod.
  c3_backlog     the same cluster under load (rho ~ 1.1 of the RAM-bound capacity):
                 pods of 0.3-0.5 of a node's RAM staying ~1,500 s, so attempts fail, pods wait in the
                 unschedulable map and are moved back to the action queue on every pod finish
                 (move-all: the conditional move is off, so the 300-s flush rarely finds an entry).
  c5             BASELINE configs[4]: the c3 replicas with the scheduler-parameter sweep of
                 workloads.c5_params (cycle interval x conditional move x network delays x CA
                 threshold x HPA tolerance; replica r of the job gets cell r), weak-scaled over the
                 ranks (8 x 8,192 = 65,536 replicas on 8 GPUs).  The c3 cluster has no autoscaler,
                 so the last two axes are inert here: see c5_autoscaled.
  c5_autoscaled  the same sweep over workloads.c5_autoscaled_parts: the 4,096-node cluster with the
                 cluster autoscaler of src/config.yaml:14-33 and the test_hpa pod group live, 16,384
                 pods of which 48 need the CA's 256-GiB template, in two bursts (the CA scales up for
                 each and back down when they drain).
A step simulates every replica from initialize() until RunUntilAllPodsAreFinished stops it.
Replicas are sharded over ranks with distinct seeds (weak scaling: R per GPU); nothing is exchanged
while they run; at the end one RCCL all-reduce of the int64 counter vector (+ the estimator rows and
histograms, all-gathered / all-reduced) combines them.

`python bench.py --gpus N`: with N > 1 and no WORLD_SIZE in the environment this process (which has
not touched the GPU) starts N rank processes of itself with RANK/LOCAL_RANK/WORLD_SIZE set, one per
GPU, and exits with their status; under torch.distributed.run WORLD_SIZE must equal N.

Prints ONE JSON line (rank 0).  `value` = placements of all ranks / max-over-ranks wall time of
the timed steps.  `roofline`: the dominant kernel is k10s_run_kernel (the whole event loop incl. the
scheduling scans); its bytes per launch are the bytes it reads for the scans (8 B per node-cache
entry read, `nodes_read`, + 12 B per attempt + 8 B per placement; roofline() below), divided by the
launch's HIP-event time measured on the engine's stream, against the 8 TB/s HBM3E peak.  SURVEY.md
§8(d)'s 12 B per node per attempt of the serial reference is reported beside it as a work rate
(`survey_pricing`), and `traffic` is the PMC-measured HBM bytes of the same build when committed.
`cpu_baseline`: the repo's CPU oracle (a string-keyed restatement of the reference, kind "port";
the Rust reference cannot be built here), one process per usable host core, each running one
replica of the same workload to completion.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12  # MI355X HBM3E peak, MI355X_MICROARCH.md "Chip-level parameters"
METRIC = "pod placements/sec (whole node, 1/2/4/8 GPUs) at 4k-node clusters; % HBM roofline"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("c3", "c3_backlog", "c5", "c5_autoscaled"), default="c3")
    ap.add_argument("--replicas", type=int, default=8192, help="replicas per GPU")
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--pods", type=int, default=16384)
    ap.add_argument("--arrival-window", type=float, default=1200.0)
    ap.add_argument("--budget", type=int, default=0, help="max events per replica per launch (0 = one launch)")
    ap.add_argument("--cpu-seconds", type=float, default=90.0,
                    help="wall-time cap per CPU-baseline replica (a replica that hits it is extrapolated)")
    ap.add_argument("--cpu-workers", type=int, default=0, help="0 = the usable host cores (cgroup quota / affinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-scan-kernel", action="store_true", help="skip the scheduling-kernel-alone measurement")
    ap.add_argument("--backlog-steps", type=int, default=3, help="timed launches of the backlog side line")
    ap.add_argument("--no-backlog-line", action="store_true",
                    help="skip the one-launch c3_backlog measurement reported beside a c3 run")
    ap.add_argument("--pruned-scan", action="store_true", help="exact block-bound pruned scan (DESIGN.md §3)")
    ap.add_argument("--delay-fifo", type=int, default=0,
                    help="entries per delay-class event ring (k10s_capacities.delay_fifo; 0 = engine default)")
    ap.add_argument("--score-plugins", choices=("least", "most", "both"), default="least",
                    help="score plugins of every replica (k10s_replica_params.score_plugins): LeastAllocated "
                         "(the reference's only one), MostAllocated (extension), or both (weights 1 and 1)")
    ap.add_argument("--replica-rows", action="store_true", help="add every replica's counters/estimators (tests)")
    ap.add_argument("--profile", action="store_true", help="print the K10S_PROF cycle attribution (variant builds)")
    ap.add_argument("--selftest-host", action="store_true",
                    help="TEST ONLY: run the launcher and the cross-rank reduction on CPU (gloo) over the "
                         "test-only host-check build; the numbers are not a measurement")
    return ap.parse_args()


# ---- N-rank launcher ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Start n rank processes of this script (one per GPU) and return the worst exit status.  The
    parent never initialises the GPU (an exec/fork after GPU init is unsafe), it only waits.  It
    brings the engine library up to date first (hipcc only, no GPU), so the ranks never compile,
    let alone concurrently; build() also serializes on a file lock for launchers other than this one
    (torch.distributed.run)."""
    from kubernetriks_amd.build import build
    build()
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        log(f"[launcher] rank exit codes {rcs}")
    return bad[0] if bad else 0


# ---- CPU baseline (oracle, one process per usable core) -----------------------------------------
def host_cores():
    """(usable cores, description): the cgroup CPU quota when there is one, else the affinity set."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(math.ceil(int(q) / int(period))))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    return usable, {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota}


def cpu_worker(args_tuple):
    """One core: the oracle runs one replica's materialized trace from t=0 until
    RunUntilAllPodsAreFinished (or the wall cap)."""
    scn, cap = args_tuple
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bridge as ob
    o = ob.OracleSim(scn)
    t0 = time.perf_counter()
    done = False
    t_sim = 0.0
    while time.perf_counter() - t0 < cap:
        t_sim += 100.0
        o.step_until_time(t_sim)
        r = o.result()
        if r["panicked"] or r["counters"]["terminated_pods"] >= r["counters"]["total_pods_in_trace"]:
            done = True
            break
        if t_sim > 1e7:
            break
    if done:  # finish exactly as the engine does (the %1000 stop rule)
        o.run_until_all_finished(1e7)
    wall = time.perf_counter() - t0
    r = o.result()
    c = r["counters"]
    return c["placements"], c["attempts"], c["events"], wall, r["time"], done, c["terminated_pods"], \
        c["total_pods_in_trace"]


def cpu_baseline(args, cfg, cluster, workload, params):
    from multiprocessing import get_context
    from kubernetriks_amd import workloads as wl
    usable, cores_info = host_cores()
    workers = args.cpu_workers or usable
    # replica i's own scenario: its parameter cell (sweeps) and its seed-perturbed trace
    jobs = [(wl.replica_scenario(cfg, cluster, workload, params[i % len(params)]), args.cpu_seconds)
            for i in range(workers)]
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bridge as ob
    ob.build_oracle()
    with get_context("fork").Pool(workers) as pool:
        res = pool.map(cpu_worker, jobs)
    rate = sum(p / w for p, _, _, w, *_ in res)
    n_done = sum(1 for r in res if r[5])
    horizon = max(r[4] for r in res)
    frac = sum(r[6] / max(r[7], 1) for r in res) / len(res)
    how = ("each run from t=0 to RunUntilAllPodsAreFinished (the whole simulated horizon, up to "
           f"t={horizon:.0f} s)") if n_done == len(res) else \
        (f"{n_done}/{len(res)} run to RunUntilAllPodsAreFinished, the others stopped at the {args.cpu_seconds:.0f} s "
         f"wall cap (on average {100 * frac:.0f}% of the pods terminated; their rate is extrapolated from that prefix)")
    sample = (f"{workers} processes (host: nproc {cores_info['nproc']}, affinity {cores_info['affinity']}, "
              f"cgroup CPU quota {cores_info['cgroup_cpu_quota']}) x 1 seed-perturbed replica each of the same "
              f"{args.workload} workload ({args.nodes} nodes, {args.pods} pods), {how}; "
              f"{sum(r[0] for r in res)} placements, {sum(r[1] for r in res)} attempts, "
              f"{sum(r[2] for r in res)} events in total")
    return {"value": rate, "unit": "placements/s", "cores": workers, "kind": "port", "sample": sample,
            "host": cores_info, "replicas_completed": n_done,
            "per_core_placements_per_s": rate / workers,
            "attempts_per_s": sum(a / w for _, a, _, w, *_ in res),
            "events_per_s": sum(e / w for _, _, e, w, *_ in res)}


# ---- the measurement ------------------------------------------------------------------------------
def pmc_traffic(workload, R, nodes, pods, pruned, score_plugins, engine):
    """HBM bytes per launch of k10s_run_kernel from the committed rocprofv3 PMC summary of this
    workload (profiles/pmc_run_kernel.json for c3, pmc_run_kernel_<workload>.json otherwise;
    tools/pmc_summary.py), only if it was taken on this exact engine build, config, scan mode and
    score plugins; else None."""
    name = "pmc_run_kernel.json" if workload == "c3" else f"pmc_run_kernel_{workload}.json"
    try:
        pm = json.load(open(os.path.join(REPO, "profiles", name)))
    except Exception:
        return None
    if pm.get("config") == [R, nodes, pods] and pm.get("engine") == engine and \
            pm.get("workload", "c3") == workload and pm.get("scan_mode") == ("pruned" if pruned else "full") and \
            pm.get("score_plugins", "least") == score_plugins:
        return pm.get("hbm_bytes_per_launch")
    return None


def roofline(entry_b, extra_b, scanned, nread, attempts, placements, launches, kernel_ms, traffic):
    """The `roofline` object of k10s_run_kernel, per launch.  `achieved` / `frac` count the bytes the
    kernel reads and writes for the scans: per node-cache entry READ (nodes_read: every scanned node,
    plus the cycle tiles' shared fit passes, whose failed attempts read no entry of their own; with the
    per-block fronts the front slots, the rebuilt blocks and the overflowing blocks) the
    entry's size (8 B packed cpu << 40 | ram, 12 B wide u32 + u64; + 12 B of capacity for
    MostAllocated), 12 B per attempt (the pod's request) and one entry per placement (the
    reservation).  `survey_pricing` is SURVEY.md 8(d)'s algorithmic volume of the serial reference
    (12 B per node per attempt, whether read or not) over the same time: a work rate, not a bandwidth
    (it exceeds the HBM peak when the tiles skip the failed attempts' scans).  `traffic`: HBM bytes per
    launch from the committed rocprofv3 PMC pass on this build, else None."""
    sec = kernel_ms * 1e-3 if kernel_ms > 0 else float("inf")
    read = ((entry_b + extra_b) * nread + 12.0 * attempts + entry_b * placements) / launches
    survey = ((12.0 + extra_b) * scanned + 12.0 * attempts + 12.0 * placements) / launches
    return {"bound": "hbm", "achieved": read / sec / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": read / sec / HBM_PEAK, "traffic": traffic,
            "traffic_frac": (traffic / sec / HBM_PEAK) if traffic else None,
            "kernel": "k10s_run_kernel", "kernel_ms_per_launch": kernel_ms,
            "bytes_per_launch": read, "node_entry_bytes": int(entry_b),
            "pricing": (f"bytes read: {int(entry_b + extra_b)} B per node-cache entry read (nodes_read) + 12 B per "
                        f"attempt + {int(entry_b)} B per placement"),
            "note": ("the per-block Pareto fronts (DESIGN.md section 3) read a fraction of the node cache per "
                     "placement, so the priced bytes and frac fall as the kernel gets faster; it is bound by each "
                     "replica's chain of dependent memory round trips, not by bandwidth (traffic_frac, DESIGN.md "
                     "section 6)"),
            "survey_pricing": {"bytes_per_launch": survey, "equivalent_GBps": survey / sec / 1e9,
                               "note": "SURVEY.md 8(d): 12 B per node per attempt + 12 B per attempt + 12 B per "
                                       "placement of the serial reference; a work rate, not a bandwidth"}}


def build_workload(args):
    """(config, cluster trace, workload trace, description, sweep) of the selected workload."""
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.scenario import SimulationConfig
    cfg, sweep = SimulationConfig(), False
    if args.workload == "c3_backlog":
        cluster, workload = wl.c3_backlog_traces(args.nodes, args.pods, args.arrival_window)
        desc = (f"C3 backlog: {args.replicas} replicas/GPU x {args.nodes}-node Alibaba-like cluster, {args.pods} pods/replica "
                "of 0.3-0.5 node RAM for ~1500 s (rho ~ 1.1 of the RAM-bound capacity: failed attempts, unschedulable "
                "map, move-all on every pod finish; conditional move off), run until all pods finished "
                "(RunUntilAllPodsAreFinished)")
    elif args.workload == "c5_autoscaled":
        cfg, cluster, workload = wl.c5_autoscaled_parts(args.nodes, args.pods, arrival_window=args.arrival_window)
        sweep = True
        desc = (f"C5 sweep with autoscalers live: {args.replicas} replicas/GPU x {args.nodes}-node Alibaba-like cluster + "
                "cluster autoscaler (config.yaml:14-33, max 200 nodes) + HPA pod group (test_hpa.rs), "
                f"{args.pods} pods/replica (48 that only the CA's 256-GiB template fits, in two bursts); replica r of the job runs "
                "cell r of workloads.c5_params (cycle interval {1,5,10,30} x conditional move {F,T} x delays "
                "x{0.5,1,2} x CA threshold {0.3,0.5,0.7} x HPA tolerance {0.05,0.1,0.2}); run until all pods finished")
    else:
        cluster, workload = wl.c3_traces(args.nodes, args.pods, args.arrival_window)
        if args.workload == "c5":
            sweep = True
            desc = (f"C5 sweep: {args.replicas} replicas/GPU x {args.nodes}-node Alibaba-like cluster, {args.pods} "
                    "pods/replica (the c3 trace, rho ~ 0.007); replica r of the job runs cell r of workloads.c5_params "
                    "(cycle interval x conditional move x delays live; CA threshold / HPA tolerance inert without "
                    "autoscalers: see c5_autoscaled); run until all pods finished")
        else:
            desc = (f"C3: {args.replicas} replicas/GPU x {args.nodes}-node Alibaba-like cluster, {args.pods} pods/replica "
                    "(rho ~ 0.007 of the RAM-bound capacity), run until all pods finished (RunUntilAllPodsAreFinished)")
    return cfg, cluster, workload, desc, sweep


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(world_env or "1")
    if world != args.gpus:
        log(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist

    from kubernetriks_amd import ensemble
    from kubernetriks_amd.native import NUM_COUNTERS, Capacities
    from kubernetriks_amd.scenario import SimulationConfig, scenario_bulk

    if args.selftest_host:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from hostcheck_bridge import HostEngine as EngineCls  # test-only build, no GPU
        backend, version = "gloo", (lambda: "host-check selftest (not a measurement)")

        def make_engine(scn, R, params=None, caps=None, blob=None):
            return EngineCls(scn, R, params=params, caps=caps, pods_blob=blob)
    else:
        from kubernetriks_amd.build import build
        build()
        from kubernetriks_amd.native import Engine, version
        backend = "nccl"
        torch.cuda.set_device(local_rank)

        def make_engine(scn, R, params=None, caps=None, blob=None):
            return Engine(scn, R, params=params, caps=caps, device=local_rank, pods_blob=blob)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
        else:
            dist.init_process_group("gloo")

    cfg, cluster, workload, desc, sweep = build_workload(args)
    # cluster trace as text, the create_pod events as the binary block (k10s_engine_create_bulk)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    R = args.replicas
    probe = make_engine(scn, 1, blob=blob)
    defaults = probe.default_params()
    del probe
    # replicas [rank*R, (rank+1)*R) of the job: seed-perturbed copies, or sweep cells (C5)
    params = ensemble.shard_params(defaults, R, rank, base_seed=123, perturb=True, sweep=sweep)
    plugins = {"least": 1, "most": 2, "both": 3}[args.score_plugins]
    for p in params:
        p.score_plugins = plugins
        if plugins & 2 and p.most_allocated_weight == 0.0:
            p.most_allocated_weight = 1.0
    t = time.perf_counter()
    caps = Capacities()
    caps.pruned_scan = 1 if args.pruned_scan else 0
    caps.delay_fifo = args.delay_fifo
    eng = make_engine(scn, R, params=params, caps=caps, blob=blob)
    log(f"[rank {rank}] engine: {R} replicas x {eng.replica_bytes / 2**20:.1f} MiB, init {time.perf_counter() - t:.2f}s")

    def one_step():
        if hasattr(eng, "reset"):
            eng.reset()
        return eng.run_until_all_finished(max_time=1e7, max_events_per_launch=args.budget)

    for i in range(args.warmup):
        t = time.perf_counter()
        one_step()
        log(f"[rank {rank}] warmup {i}: {time.perf_counter() - t:.2f}s")

    counters = np.zeros(NUM_COUNTERS, dtype=np.int64)
    kernel_ms = []
    if world > 1:
        dist.barrier()
    if backend == "nccl":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ms = one_step()
        kernel_ms.append(ms)
        counters += eng.counter_matrix().sum(axis=0, dtype=np.uint64).astype(np.int64)
        log(f"[rank {rank}] step {i}: run {ms:.1f} ms")
    if backend == "nccl":
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

    # cross-rank reduction (RCCL over xGMI): max of the timings, int64 sum of the counters; the
    # per-replica estimators of the last step are gathered in rank order into the job's ensemble summary
    elapsed, mean_kernel_ms = ensemble.max_over_ranks([elapsed, sum(kernel_ms) / max(len(kernel_ms), 1)])
    c = ensemble.sum_over_ranks(counters.tolist())
    summary = ensemble.ensemble_summary(eng.raw_results()).as_dict()
    st_all = ensemble.sum_over_ranks([statuses.get(s, 0) for s in range(5)])  # replica status histogram, all ranks
    statuses = {s: n for s, n in enumerate(st_all) if n}
    placements, attempts, events, scanned, nread = c[12], c[13], c[14], c[15], c[16]
    value = placements / elapsed

    # roofline for the dominant kernel (per launch, this rank's launch time, all-rank bytes / world)
    traffic = None if args.selftest_host else pmc_traffic(args.workload, R, args.nodes, args.pods, args.pruned_scan,
                                                            args.score_plugins, version())
    roof = roofline(float(eng.node_entry_bytes), 0.0 if args.score_plugins == "least" else 12.0, scanned, nread,
                    attempts, placements, args.steps * world, mean_kernel_ms, traffic)
    roof["scan_mode"] = "pruned" if args.pruned_scan else "full"
    entry_b = float(eng.node_entry_bytes)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "placements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / max(args.steps, 1) * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: Alibaba-like 4096-node clusters and 16384-pod traces (notebook statistics), "
                 "seed-perturbed per replica") if not args.selftest_host else "selftest (host-check build on CPU)",
        "config": {"workload": desc, "workload_name": args.workload,
                   "replicas_per_gpu": R, "total_replicas": R * world, "nodes": args.nodes, "pods_per_replica": args.pods,
                   "score_plugins": args.score_plugins, "node_entry_bytes": int(entry_b),
                   "parallelism": f"replica-sharded x{world} (RCCL all-reduce of counters and histograms only)"},
        "roofline": roof,
        "engine": version(),
        "rates": {"placements_per_s": value, "attempts_per_s": attempts / elapsed, "events_per_s": events / elapsed},
        "totals": {"placements": placements, "attempts": attempts, "events": events, "nodes_scanned": scanned,
                   "nodes_read": nread,
                   "replica_status": {str(k): v for k, v in statuses.items()}, "replica_errors": errors},
        "ensemble": {"replicas": summary["replicas"], "replica_status": summary["replica_status"],
                     "counters": {k: summary["counters"][k] for k in ("total_pods_in_trace", "pods_succeeded",
                                                                       "terminated_pods", "placements", "attempts",
                                                                       "events")},
                     "timings": summary["timings"], "histograms": summary.get("histograms")},
    }
    if args.replica_rows:   # per-replica fingerprints in global replica order (tests of the rank sharding)
        rc, re_, rs = ensemble.gather_rows(eng.raw_results())
        out["replica_rows"] = {"counters": rc.tolist(), "estimators": re_.reshape(len(rc), -1).tolist(),
                               "status": rs.tolist()}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args, cfg, cluster, workload, params)
        except Exception as ex:  # the GPU number stands on its own
            log("cpu baseline failed:", ex)
            out["cpu_baseline"] = None
    if rank == 0 and not args.no_scan_kernel and not args.selftest_host:
        # the scheduling-cycle kernel alone (k10s_schedule_one_batch over C3-sized node caches in HBM)
        try:
            from kubernetriks_amd.scanbench import measure
            out["scheduling_kernel"] = measure(R, args.nodes)
        except Exception as ex:
            log("scan kernel measurement failed:", ex)
            out["scheduling_kernel"] = None
    if args.profile:
        prof = eng.profile()
        scal = [k for k in prof[0] if not k.startswith("kind_")]
        tot = {k: float(sum(p[k] for p in prof)) for k in scal}
        loop = tot["loop"] or 1.0
        out["profile"] = {"cycles_total": tot, "share_of_loop": {k: v / loop for k, v in tot.items() if not k.startswith("n")
                                                                 and k != "scans"},
                          "cycles_per_event": loop / max(events / args.steps / world, 1.0),
                          "scan_cycles_per_scan": tot["scan"] / max(tot["scans"], 1.0)}
        if "kind_cycles" in prof[0]:
            from kubernetriks_amd.native import EVENT_KIND_NAMES
            kc = [sum(p["kind_cycles"][k] for p in prof) for k in range(len(prof[0]["kind_cycles"]))]
            kn = [sum(p["kind_count"][k] for p in prof) for k in range(len(prof[0]["kind_count"]))]
            out["profile"]["by_kind"] = {EVENT_KIND_NAMES.get(k, str(k)): {"count": kn[k], "share_of_loop": kc[k] / loop,
                                                                         "cycles_per_event": kc[k] / max(kn[k], 1)}
                                         for k in range(len(kc)) if kn[k]}
    if rank == 0 and world == 1 and args.workload == "c3" and args.score_plugins == "least" and not args.no_backlog_line and not args.selftest_host:
        # the same replicas under load (failed attempts, unschedulable map, move-all on every finish): one launch
        try:
            del eng
            out["backlog"] = backlog_line(args, cfg, make_engine, caps, ensemble, NUM_COUNTERS, version)
        except Exception as ex:
            log("backlog measurement failed:", ex)
            out["backlog"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def backlog_line(args, cfg, make_engine, caps, ensemble, num_counters, version):
    """One launch of the c3_backlog workload (same replica count, nodes and pods) beside a c3 run, so
    the default bench line also shows the regime where attempts fail.  Not the headline value."""
    import argparse
    import numpy as np
    import torch
    from kubernetriks_amd.scenario import scenario_bulk
    b = argparse.Namespace(**vars(args))
    b.workload = "c3_backlog"
    cfg, cluster, workload, desc, _ = build_workload(b)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    probe = make_engine(scn, 1, blob=blob)
    defaults = probe.default_params()
    del probe
    params = ensemble.shard_params(defaults, args.replicas, 0, base_seed=123, perturb=True)
    eng = make_engine(scn, args.replicas, params=params, caps=caps, blob=blob)
    steps, warmup = args.backlog_steps, 1
    for _ in range(warmup):
        eng.reset()
        eng.run_until_all_finished(max_time=1e7)
    c = np.zeros(num_counters, dtype=np.int64)
    kms = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.reset()
        kms.append(eng.run_until_all_finished(max_time=1e7))
        c += eng.counter_matrix().sum(axis=0, dtype=np.uint64).astype(np.int64)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = sum(kms) / len(kms)
    placements, attempts, scanned, nread = int(c[12]), int(c[13]), int(c[15]), int(c[16])
    traffic = pmc_traffic("c3_backlog", args.replicas, args.nodes, args.pods, args.pruned_scan, "least", version())
    roof = roofline(float(eng.node_entry_bytes), 0.0, scanned, nread, attempts, placements, steps, ms, traffic)
    log(f"backlog: {placements / elapsed / 1e6:.2f} M placements/s, run {ms:.1f} ms")
    return {"workload": desc, "workload_name": "c3_backlog", "steps": steps, "warmup": warmup,
            "placements_per_s": placements / elapsed, "attempts_per_s": attempts / elapsed,
            "ms_per_step": elapsed * 1e3 / steps, "kernel_ms_per_launch": ms, "roofline": roof,
            "totals": {"placements": placements, "attempts": attempts, "nodes_scanned": scanned, "nodes_read": nread,
                       "requeued": int(c[17]), "flushed": int(c[18])},
            "engine": version()}


if __name__ == "__main__":
    main()
