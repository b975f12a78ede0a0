"""Runs of one event kind handled together (k10s_engine.h run_batch): parity against the oracle on
bursty scenarios built to produce them and to hit every reason a run is refused.

A run is the next K events in dslab order from one source, of one kind, at one time.  The scenarios
below put many pods (and nodes) at few distinct times: arrival bursts (AS_CREATE_POD_REQ from the
trace, then PS_CREATE_POD_REQ and S_POD_SCHEDULE_REQ from the rings), node-creation bursts (the five
kinds of the node chain, the api server's answer on the same ring as storage's request), node
removals and re-creations in bursts, pods that wait in the unschedulable map when nodes arrive
(S_ADD_NODE runs refused), bursts interleaved with other sources at the same time (the run stops at
the second source's head), tiny delay rings (full rings refuse runs), budgeted launches that cut runs,
step_until_time checkpoints, pod groups and the cluster autoscaler.  Every replica is compared with the
oracle bit for bit, event log included.
"""
import ctypes
import os
import random
import subprocess

import pytest

import oracle_bridge as ob
import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED, RUN_UNTIL_TIME
from kubernetriks_amd.scenario import (CANodeGroup, DefaultNodeGroup, GenericClusterTrace, GenericWorkloadTrace,
                                       Node, Pod, PodGroup, SimulationConfig, UsageModel, WorkloadEvent,
                                       scenario_text, test_simulation_config)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpu_engine():
    from kubernetriks_amd.native import Engine
    return Engine


BACKENDS = [
    pytest.param("host", id="host"),
    pytest.param("gpu", id="gpu", marks=pytest.mark.gpu),
]


def engine_cls(backend):
    return HostEngine if backend == "host" else _gpu_engine()


def bursty_scenario(seed: int, n_pods: int = 240, n_nodes: int = 40) -> str:
    rng = random.Random(seed)
    cfg = test_simulation_config() if rng.random() < 0.5 else SimulationConfig()
    cfg.enable_unscheduled_pods_conditional_move = rng.random() < 0.3
    cfg.scheduling_cycle_interval = rng.choice([1.0, 5.0, 10.0])
    if rng.random() < 0.3:
        cfg.default_cluster = [DefaultNodeGroup(rng.randint(1, 3), Node("", 8000, 16 << 30))]
    times = sorted({float(rng.randint(0, 400)) for _ in range(rng.randint(3, 8))})
    node_times = [0.0] + [t for t in times if rng.random() < 0.4]
    cluster = GenericClusterTrace()
    alive = {}
    for i in range(n_nodes):
        nm = f"node_{i:03d}"
        t = rng.choice(node_times) if rng.random() < 0.8 else float(rng.randint(0, 400))
        cpu = rng.choice([4000, 8000, 16000])
        ram = rng.choice([8 << 30, 16 << 30, 32 << 30])
        cluster.create_node(t, Node(nm, cpu, ram))
        alive[nm] = t
    if seed % 10 == 3:   # one node created twice in its burst: the reference panics in storage
        nm = next(iter(alive))
        cluster.create_node(alive[nm], Node(nm, 4000, 8 << 30))
    if rng.random() < 0.5:   # a burst of removals, half of them re-created in a later burst
        t_rm = max(node_times) + float(rng.randint(50, 200))
        t_re = t_rm + float(rng.randint(1, 100))
        for nm in list(alive)[: n_nodes // 3]:
            cluster.remove_node(t_rm, nm)
            if rng.random() < 0.5:
                cluster.create_node(t_re, Node(nm, 8000, 16 << 30))
    workload = GenericWorkloadTrace()
    names = []
    for i in range(n_pods):
        r = rng.random()
        if r < 0.05:
            cpu, ram = 40000, 1 << 30   # never fits: waits in the unschedulable map
        else:
            cpu = rng.choice([250, 500, 1000, 2000])
            ram = rng.choice([1 << 29, 1 << 30, 2 << 30])
        dur = float(rng.randint(1, 300))
        t = rng.choice(times)
        if rng.random() < 0.15:
            t = -1.0   # placeholder: before any node (pods wait when the nodes arrive)
        name = f"pod_{i:04d}"
        workload.create_pod(max(t, 0.0), Pod(name, cpu, ram, dur))
        names.append(name)
    for name in names:
        if rng.random() < 0.05:
            workload.remove_pod(rng.choice(times) + float(rng.randint(0, 3)), name)
    if rng.random() < 0.3:
        cfg.hpa_enabled = True
        cfg.hpa_scan_interval = 30.0
        g = PodGroup("group_0", rng.randint(2, 8), rng.randint(8, 20), Pod("group_0", 100, 100 << 20, None), 0.6,
                     None, UsageModel("pod_group", units=[(200.0, 8.0), (100.0, 2.0)]), None)
        workload.events.append(WorkloadEvent(rng.choice(times), "create_pod_group", pod_group=g))
    if rng.random() < 0.25:
        cfg.ca_enabled = True
        cfg.ca_max_node_count = 4
        cfg.ca_scan_interval = 10.0
        cfg.ca_node_groups = [CANodeGroup("ca_big", None, 16000, 32 << 30)]
    return scenario_text(cfg, cluster, workload)


def _mode(scn):
    return RUN_UNTIL_TIME if "hpa_config enabled 1" in scn else RUN_UNTIL_ALL_FINISHED


SEEDS_HOST = list(range(40))
SEEDS_GPU = list(range(40))


def _case(backend, seed, fifo=0, budget=0):
    scn = bursty_scenario(seed)
    od, eng = parity.run_pair(engine_cls(backend), scn, mode=_mode(scn), until=2000.0, max_time=20000.0,
                              fifo=fifo, budget=budget)
    assert parity.compare(od, eng) == [], (seed, fifo, budget)


@pytest.mark.parametrize("seed", SEEDS_HOST)
def test_bursty_host(seed):
    _case("host", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS_GPU)
def test_bursty_gpu(seed):
    _case("gpu", seed)


# tiny rings (a run that does not fit goes event by event, as do its emissions to the heap) and
# budgeted launches (a budget cuts a run; the next launch resumes inside it)
LIMIT_CASES = [(s, fifo, budget) for s in (1, 2, 5, 7) for fifo, budget in ((2, 0), (4, 0), (0, 1), (0, 3), (8, 37))]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed,fifo,budget", LIMIT_CASES)
def test_bursty_ring_and_budget_limits(backend, seed, fifo, budget):
    _case(backend, seed, fifo, budget)


@pytest.mark.parametrize("backend", BACKENDS)
def test_bursty_stepping_matches_oracle(backend):
    """step_until_time checkpoints at and just before burst times (a run is never split by a
    checkpoint: its events share one time)."""
    scn = bursty_scenario(11)
    o = ob.OracleSim(scn, log=True, gauges=parity.GAUGE_ROWS)
    eng = engine_cls(backend)(scn, 2, caps=parity.parity_caps(True, gauges=parity.GAUGE_ROWS))
    for t in (0.0, 5.0, 99.999, 100.0, 250.0, 400.0, 1000.0):
        o.step_until_time(t)
        eng.step_until_time(t)
        od = o.result(placements=True, log=True)
        od["status_name"] = "running" if not od["panicked"] else "error"
        for r in range(2):
            assert parity.compare(od, eng, r=r) == [], (t, r)


_STATS = {}


def _stats_lib():
    """The host build with event-path statistics (tools/host_stats.py's build), compiled once per
    test process (per-process file name: pytest-xdist workers build side by side)."""
    if "lib" not in _STATS:
        tag = os.getpid()
        out = os.path.join(REPO, "build", f"libk10s_hoststats_runs_{tag}.so")
        defs = os.path.join(REPO, "build", f"hoststats_runs_defs_{tag}.cpp")
        with open(defs, "w") as f:
            f.write('#include <cstdint>\nextern "C" uint64_t k10s_host_stats[48];\nuint64_t k10s_host_stats[48];\n')
        hc = os.path.join(REPO, "tests", "hostcheck")
        subprocess.check_call(["g++", "-O1", "-std=c++17", "-fPIC", "-ffp-contract=off", "-DK10S_HOST_STATS", "-shared",
                               "-o", out, os.path.join(hc, "hostcheck.cpp"),
                               os.path.join(REPO, "kubernetriks_amd", "csrc", "k10s_builder.cpp"), defs])
        os.unlink(defs)
        _STATS["lib"] = out
        import atexit
        atexit.register(lambda: os.path.exists(out) and os.unlink(out))
    return _STATS["lib"]


def test_runs_cover_the_bursts():
    """On a bursty scenario most events go through runs (host build with event statistics)."""
    out = _stats_lib()
    L = ctypes.CDLL(out)
    import hostcheck_bridge as hb
    saved = (hb.LIB_PATH, hb._lib, hb.build)
    try:
        hb.LIB_PATH, hb._lib, hb.build = out, None, (lambda: None)
        from kubernetriks_amd import workloads as wl
        cluster, workload = wl.c3_traces(n_nodes=256, n_pods=1024, arrival_window=100.0, seed=3)
        eng = hb.HostEngine(scenario_text(SimulationConfig(), cluster, workload), 1)
        eng.run_until_all_finished(max_time=1e7)
        st = (ctypes.c_uint64 * 48).in_dll(L, "k10s_host_stats")
        events, runs, run_events = int(st[0]), int(st[38]), int(st[39])
        for i in range(48):
            st[i] = 0
    finally:
        hb.LIB_PATH, hb._lib, hb.build = saved
    assert runs > 100 and run_events > 0.2 * events, (events, runs, run_events)


# ---- windows of the assignment pipeline (k10s_engine.h win_batch) -----------------------------------
def pipeline_scenario(seed: int, n_pods: int = 300) -> str:
    """Cycles that place many pods at once on few nodes: the six pipeline kinds interleave, several
    assignments per node and binds per component fall inside one window (the window must stop
    there), with zero and equal network delays (windows of equal-time events only), pod groups (the
    group's running count), pod removals (the api server's removal set), node removals while
    assignments are in flight (binds on removed nodes panic in the reference), tiny rings."""
    rng = random.Random(seed)
    cfg = test_simulation_config()
    cfg.scheduling_cycle_interval = rng.choice([5.0, 10.0, 30.0])
    d = rng.choice([0.0, 0.001, 0.05, 0.15])
    cfg.as_to_ps_network_delay = d if rng.random() < 0.5 else rng.choice([0.0, 0.02, 0.05])
    cfg.as_to_node_network_delay = d if rng.random() < 0.5 else rng.choice([0.0, 0.03, 0.15])
    cfg.sched_to_as_network_delay = rng.choice([0.0, 0.02])
    cfg.ps_to_sched_network_delay = rng.choice([0.0, 0.01, 0.089])
    cfg.enable_unscheduled_pods_conditional_move = rng.random() < 0.3
    cluster = GenericClusterTrace()
    n_nodes = rng.randint(1, 6)
    for i in range(n_nodes):
        cluster.create_node(0.0, Node(f"node_{i}", 64000, 256 << 30))
    if rng.random() < 0.5:   # a node removed (and maybe re-created) while pods are being bound to it
        t = float(rng.choice([10, 20, 30, 60])) + rng.choice([0.0, 0.02, 0.05, 0.1])
        cluster.remove_node(t, "node_0")
        if rng.random() < 0.5:
            cluster.create_node(t + 7.0, Node("node_0", 64000, 256 << 30))
    workload = GenericWorkloadTrace()
    names = []
    for i in range(n_pods):
        t = float(rng.randint(0, 120))
        name = f"pod_{i:04d}"
        workload.create_pod(t, Pod(name, rng.choice([100, 500, 1000]), rng.choice([1 << 28, 1 << 30]),
                                   float(rng.randint(0, 200)) if rng.random() < 0.9 else None))
        names.append(name)
    for name in names:
        if rng.random() < 0.04:
            workload.remove_pod(float(rng.randint(0, 150)) + rng.choice([0.0, 0.02, 0.05]), name)
    if rng.random() < 0.4:
        cfg.hpa_enabled = True
        cfg.hpa_scan_interval = 30.0
        g = PodGroup("group_0", rng.randint(3, 10), 30, Pod("group_0", 100, 100 << 20, None), 0.6, None,
                     UsageModel("pod_group", units=[(100.0, 8.0), (50.0, 1.0)]), None)
        workload.events.append(WorkloadEvent(float(rng.randint(0, 60)), "create_pod_group", pod_group=g))
    return scenario_text(cfg, cluster, workload)


PIPE_SEEDS = list(range(30))


def _pipe(backend, seed, fifo=0, gauges=0):
    scn = pipeline_scenario(seed)
    mode = _mode(scn)
    o = ob.OracleSim(scn, log=True, gauges=gauges or parity.GAUGE_ROWS)
    st = o.run_until_all_finished(20000.0) if mode == RUN_UNTIL_ALL_FINISHED else o.step_until_time(1000.0)
    od = o.result(placements=True, log=True)
    od["status_name"] = parity.ORACLE_STATUS[st] if not od["panicked"] else "error"
    caps = parity.parity_caps(True, fifo=fifo, gauges=gauges or parity.GAUGE_ROWS)
    eng = engine_cls(backend)(scn, 1, caps=caps)
    if mode == RUN_UNTIL_ALL_FINISHED:
        eng.run_until_all_finished(20000.0)
    else:
        eng.step_until_time(1000.0)
    assert parity.compare(od, eng) == [], (seed, fifo)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed", PIPE_SEEDS)
def test_pipeline_windows_match_oracle(backend, seed):
    _pipe(backend, seed)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed,fifo", [(s, f) for s in (0, 3, 8) for f in (2, 4, 16)])
def test_pipeline_windows_small_rings(backend, seed, fifo):
    _pipe(backend, seed, fifo=fifo)


def test_windows_cover_the_pipeline():
    """On the C3 shape the six pipeline kinds go through windows (host build with event statistics)."""
    out = _stats_lib()
    L = ctypes.CDLL(out)
    import hostcheck_bridge as hb
    saved = (hb.LIB_PATH, hb._lib, hb.build)
    try:
        hb.LIB_PATH, hb._lib, hb.build = out, None, (lambda: None)
        from kubernetriks_amd import workloads as wl
        st = (ctypes.c_uint64 * 48).in_dll(L, "k10s_host_stats")
        before = [int(st[i]) for i in (0, 41, 42)]
        cluster, workload = wl.c3_traces(n_nodes=256, n_pods=1024, arrival_window=100.0, seed=4)
        eng = hb.HostEngine(scenario_text(SimulationConfig(), cluster, workload), 1)
        eng.run_until_all_finished(max_time=1e7)
        events, wins, win_events = (int(st[i]) - b for i, b in zip((0, 41, 42), before))
    finally:
        hb.LIB_PATH, hb._lib, hb.build = saved
    assert wins > 20 and win_events > 0.25 * events, (events, wins, win_events)


def test_finish_relay_fused_and_refused():
    """The finish relay (k10s_engine.h finish_relay_next) is handled inside the finish when it is the
    next event, and left to the loop when another event shares or precedes its time.  Both happen on
    the bursty scenarios (integer arrivals and durations: finishes tie in time), whose parity the
    tests above check; here the host build with event statistics shows both branches ran."""
    out = _stats_lib()
    L = ctypes.CDLL(out)
    import hostcheck_bridge as hb
    saved = (hb.LIB_PATH, hb._lib, hb.build)
    try:
        hb.LIB_PATH, hb._lib, hb.build = out, None, (lambda: None)
        st = (ctypes.c_uint64 * 48).in_dll(L, "k10s_host_stats")
        before = int(st[45])
        finished = 0
        for seed in (0, 1, 2, 4, 5):
            scn = bursty_scenario(seed)
            eng = hb.HostEngine(scn, 1)
            if _mode(scn) == RUN_UNTIL_TIME:
                eng.step_until_time(2000.0)
            else:
                eng.run_until_all_finished(max_time=20000.0)
            finished += eng.results()[0]["counters"]["pods_succeeded"]
        fused = int(st[45]) - before
    finally:
        hb.LIB_PATH, hb._lib, hb.build = saved
    assert 0 < fused < finished, (fused, finished)


def gauge_straddle_scenario(seed: int) -> str:
    """windows next to the gauge recorder.  Network delays of 1.2-2.6 s make every
    cycle's assignment pipeline span several 5-s gauge ticks (M_GAUGE_TICK, a heap event and not a
    window kind), and the node-component binds (the gauge's per-slot allocatable, N_BIND) and the
    storage assignments of a window land on both sides of a tick: a window that ran across a tick, or
    applied its binds in another order, would change a gauge row (node averages summed in name order,
    cluster sums) against the oracle."""
    rng = random.Random(seed)
    cfg = test_simulation_config()
    cfg.scheduling_cycle_interval = rng.choice([5.0, 7.0])
    cfg.as_to_ps_network_delay = rng.choice([1.2, 1.9, 2.5])
    cfg.as_to_node_network_delay = rng.choice([1.3, 2.6])
    cfg.sched_to_as_network_delay = rng.choice([0.4, 1.1])
    cfg.ps_to_sched_network_delay = 0.3
    cluster = GenericClusterTrace()
    for i in range(rng.randint(3, 12)):
        cluster.create_node(0.0, Node(f"node_{i:02d}", rng.choice([16000, 64000]), rng.choice([64, 256]) << 30))
    workload = GenericWorkloadTrace()
    for i in range(400):
        workload.create_pod(float(rng.randint(0, 200)) + rng.choice([0.0, 0.5, 4.9]),
                            Pod(f"pod_{i:04d}", rng.choice([100, 500, 3000]), rng.choice([1 << 28, 1 << 30, 8 << 30]),
                                float(rng.randint(1, 60))))
    return scenario_text(cfg, cluster, workload)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed", range(6))
def test_windows_keep_gauge_rows_exact(backend, seed):
    scn = gauge_straddle_scenario(seed)
    od, eng = parity.run_pair(engine_cls(backend), scn, max_time=20000.0)
    assert parity.compare(od, eng) == [], seed
    assert len(eng.gauges(0)) > 20


def test_gauge_straddle_scenarios_use_windows():
    """The gauge-straddle scenarios above do run windows (host build with event statistics)."""
    out = _stats_lib()
    L = ctypes.CDLL(out)
    import hostcheck_bridge as hb
    saved = (hb.LIB_PATH, hb._lib, hb.build)
    try:
        hb.LIB_PATH, hb._lib, hb.build = out, None, (lambda: None)
        st = (ctypes.c_uint64 * 48).in_dll(L, "k10s_host_stats")
        for seed in range(6):
            before = [int(st[i]) for i in (0, 41, 42)]
            eng = hb.HostEngine(gauge_straddle_scenario(seed), 1)
            eng.run_until_all_finished(max_time=20000.0)
            events, wins, win_events = (int(st[i]) - b for i, b in zip((0, 41, 42), before))
            assert wins > 100 and win_events > 0.25 * events, (seed, events, wins, win_events)
    finally:
        hb.LIB_PATH, hb._lib, hb.build = saved
