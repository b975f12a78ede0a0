"""Cluster-autoscaler decisions (kube_cluster_autoscaler.rs:62-326) engine vs oracle, on scenarios
built to exercise what the lane-parallel device decision does differently from the reference's
loops (k10s_engine.h ca_decide):

  * the unscheduled-pod cache read as a bitmap in name order (scale_up, 191-245), with the panic of
    scale_up_info on a removed cached pod (persistent_storage.rs:137-145) kept as a counter;
  * CA nodes holding more than 64 pods, so a node's assignment list is gathered and rank-sorted by
    name in several 64-lane passes (all_pods_can_be_moved_to_other_nodes, 148-181);
  * first-fit over more than 256 node-cache entries (4-node lane groups, several steps), zero-request
    pods (they fit any other PS node), node removal and re-creation of CA names;
  * the BASELINE C5 shape with its autoscaler axes live (workloads.c5_autoscaled_parts): 4,096
    Alibaba-like nodes, a burst of pods only the CA's 256-GiB template fits, an HPA pod group, and
    the parameter sweep of workloads.c5_params.
Every compared replica is bit-exact with the oracle (counters incl. scaled up/down nodes and pods,
estimators, clock, placements, per-pod times)."""
import random

import pytest

import oracle_bridge as ob
import oracle_jobs
import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd import workloads as wl
from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED
from kubernetriks_amd.scenario import (CANodeGroup, GenericClusterTrace, GenericWorkloadTrace, Node, Pod,
                                       SimulationConfig, scenario_text)


def engine_cls(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


def ca_stress_scenario(seed: int, n_trace: int = 40, n_pods: int = 500, max_nodes: int = 20) -> str:
    """Small trace nodes that a burst of small pods overflows: the CA scales up big nodes, the pods
    that land there (LeastAllocated prefers the empty CA node) are many per node, and as the burst
    drains the CA tries to move them back onto the trace nodes before removing the node."""
    rng = random.Random(seed)
    cfg = SimulationConfig()
    cfg.scheduling_cycle_interval = rng.choice([1.0, 5.0, 10.0])
    cfg.enable_unscheduled_pods_conditional_move = rng.random() < 0.4
    cfg.ca_enabled = True
    cfg.ca_max_node_count = max_nodes
    cfg.ca_scan_interval = rng.choice([5.0, 10.0, 30.0])
    cfg.ca_scale_down_utilization_threshold = rng.choice([0.3, 0.5, 0.7, 0.9])
    cfg.ca_node_groups = [CANodeGroup("ca_big", rng.choice([None, 6]), 64000, 128 << 30),
                          CANodeGroup("ca_small", None, 8000, 16 << 30)]
    c = GenericClusterTrace()
    for k in range(n_trace):
        c.create_node(0.0, Node(f"trace_{k:03d}", rng.choice([4000, 8000]), rng.choice([8 << 30, 16 << 30])))
    if rng.random() < 0.5:   # trace nodes removed (and some re-created) while the CA runs
        for k in rng.sample(range(n_trace), 4):
            t = float(rng.randint(50, 600))
            c.remove_node(t, f"trace_{k:03d}")
            if rng.random() < 0.5:
                c.create_node(t + rng.randint(1, 300), Node(f"trace_{k:03d}", 8000, 16 << 30))
    w = GenericWorkloadTrace()
    names = []
    for i in range(n_pods):
        r = rng.random()
        if r < 0.03 and seed % 4 == 3:
            # zero request: never schedules, so it stays in the unscheduled cache and the CA never
            # scales down again (only in some seeds)
            cpu, ram = 0, 0
        elif r < 0.06:
            cpu, ram = 0, rng.randint(1, 1 << 28)
        elif r < 0.10:
            cpu, ram = 20000, 40 << 30                # only the big template fits
        else:
            cpu, ram = rng.choice([100, 200, 500, 1000]), rng.choice([1 << 27, 1 << 28, 1 << 29, 1 << 30])
        t = float(rng.randint(1, 200)) if rng.random() < 0.8 else float(rng.randint(200, 900))
        nm = f"pod_{i:04d}"
        w.create_pod(t, Pod(nm, cpu, ram, float(rng.randint(20, 700))))
        names.append(nm)
    if seed % 3 == 2:   # removals; a removed pod still in the unscheduled cache panics scale_up_info
        for nm in rng.sample(names, 10):
            w.remove_pod(float(rng.randint(5, 800)), nm)
    return scenario_text(cfg, c, w)


CA_SEEDS = list(range(12))


def _ca_case(backend, seed):
    scn = ca_stress_scenario(seed)
    # some seeds oscillate (a scale-up and a scale-down every tick): "{group}_{k}" names run past the
    # default name bound (max_node_count * 8 + 16), so the universe is widened
    od, eng = parity.run_pair(engine_cls(backend), scn, max_time=50000.0, ca_name_bound=4096)
    assert parity.compare(od, eng) == [], seed
    return eng.results()[0]["counters"], od


@pytest.mark.parametrize("seed", CA_SEEDS)
def test_ca_stress_host(seed):
    _ca_case("host", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", CA_SEEDS)
def test_ca_stress_gpu(seed):
    _ca_case("gpu", seed)


def test_ca_stress_covers_the_decision_paths():
    """The stress scenarios do what they are for (checked on the oracle's own counters): scale-ups,
    scale-downs, and CA nodes whose pods had to be moved (a node with more than 64 of them)."""
    ups = downs = panics = 0
    for seed in CA_SEEDS:
        o = ob.OracleSim(ca_stress_scenario(seed), log=True)
        o.run_until_all_finished(50000.0)
        r = o.result()
        ups += r["counters"]["total_scaled_up_nodes"]
        downs += r["counters"]["total_scaled_down_nodes"]
        panics += bool(r["panicked"])
    assert ups > 50 and downs > 50
    assert panics < len(CA_SEEDS)


def test_ca_node_with_many_pods_moves_them_in_name_order():
    """One CA node holding 150 pods (> 2 lane passes of the rank sort) under the threshold: the CA
    moves all of them onto trace nodes that free up, in name order, then removes the node."""
    cfg = SimulationConfig()
    cfg.ca_enabled = True
    cfg.ca_max_node_count = 2
    cfg.ca_scan_interval = 10.0
    cfg.ca_scale_down_utilization_threshold = 0.5
    cfg.ca_node_groups = [CANodeGroup("ca_big", None, 64000, 128 << 30)]
    c = GenericClusterTrace()
    for k in range(3):
        c.create_node(0.0, Node(f"trace_{k}", 16000, 32 << 30))
    w = GenericWorkloadTrace()
    rng = random.Random(5)
    for i in range(3):   # fill the trace nodes for a while
        w.create_pod(1.0, Pod(f"a_filler_{i}", 16000, 1 << 30, 400.0))
    order = list(range(150))
    rng.shuffle(order)     # arrival order is not name order
    for j, i in enumerate(order):
        w.create_pod(20.0 + j // 30, Pod(f"b_small_{i:03d}", 100, 64 << 20, 2000.0 + i))
    scn = scenario_text(cfg, c, w)
    for E in (HostEngine,):
        od, eng = parity.run_pair(E, scn, max_time=50000.0)
        assert parity.compare(od, eng) == []
        cnt = eng.results()[0]["counters"]
        assert cnt["total_scaled_up_nodes"] >= 1 and cnt["total_scaled_down_nodes"] >= 1


@pytest.mark.gpu
def test_ca_node_with_many_pods_gpu():
    from kubernetriks_amd.native import Engine
    cfg = SimulationConfig()
    cfg.ca_enabled = True
    cfg.ca_max_node_count = 2
    cfg.ca_scale_down_utilization_threshold = 0.5
    cfg.ca_node_groups = [CANodeGroup("ca_big", None, 64000, 128 << 30)]
    c = GenericClusterTrace()
    for k in range(3):
        c.create_node(0.0, Node(f"trace_{k}", 16000, 32 << 30))
    w = GenericWorkloadTrace()
    rng = random.Random(5)
    for i in range(3):
        w.create_pod(1.0, Pod(f"a_filler_{i}", 16000, 1 << 30, 400.0))
    order = list(range(150))
    rng.shuffle(order)
    for j, i in enumerate(order):
        w.create_pod(20.0 + j // 30, Pod(f"b_small_{i:03d}", 100, 64 << 20, 2000.0 + i))
    od, eng = parity.run_pair(Engine, scenario_text(cfg, c, w), max_time=50000.0)
    assert parity.compare(od, eng) == []


# ---- C5 with its autoscaler axes live ----------------------------------------------------------
def _c5a_check(backend, R, check, parts):
    cfg, cluster, workload = parts
    E = engine_cls(backend)
    scn = scenario_text(cfg, cluster, workload)
    params = wl.c5_params(E(scn, 1).default_params(), R, base_seed=123)
    eng = E(scn, R, params=params, caps=parity.parity_caps(False))
    eng.run_until_all_finished(1e6)
    ods = oracle_jobs.replay_many([wl.replica_scenario(cfg, cluster, workload, params[r]) for r in check], 1e6,
                                  workers=0 if backend == "gpu" else 1)
    for r, od in zip(check, ods):
        assert parity.compare(od, eng, r=r, log=False) == [], r
    return eng


def test_c5_autoscaled_small_host():
    """The c5_autoscaled workload at a CPU-sized shape: the sweep cells of the first replicas (cycle
    interval x conditional move) with the CA threshold and HPA tolerance of replicas 24/72/144."""
    parts = wl.c5_autoscaled_parts(n_nodes=48, n_pods=300, n_big=24, arrival_window=200.0)
    eng = _c5a_check("host", 3, [0, 1, 2], parts)
    c = eng.results()[0]["counters"]
    assert c["total_scaled_up_nodes"] > 0 and c["total_scaled_up_pods"] > 0


C5A_CELLS = sorted({(ci % 4) + 4 * ((ci // 4) % 2) + 24 * ((ci // 8) % 3) + 72 * (ci // 24) for ci in range(72)})


@pytest.mark.gpu
def test_c5_autoscaled_sweep_at_baseline_size_gpu():
    """One GPU's share of the C5 sweep (8,192 replicas) on 4,096-node clusters with the CA and the
    HPA live.  The oracle replays one replica of every (cycle interval x conditional move x CA
    threshold x HPA tolerance) cell of workloads.c5_params (72 cells; the delay axis at its first
    value), and the batch as a whole scales nodes and pods up and down."""
    R = 8192
    parts = wl.c5_autoscaled_parts(n_nodes=4096, n_pods=1500, n_big=100, arrival_window=300.0)
    assert len(C5A_CELLS) == 72
    eng = _c5a_check("gpu", R, C5A_CELLS, parts)
    res = eng.results()
    # Some cells hit a reference panic (an HPA scale-down removes a pod whose node the CA has just
    # scaled down: node_component.rs unwraps the reclaimed component), reproduced bit-exactly above
    # wherever a replayed cell has it; nothing else may stop a replica (no engine capacity errors)
    st = [(r["status"], r["error_code"]) for r in res]
    assert all(s == ("finished", 0) or (s[0] == "error" and 0 < s[1] < 100) for s in st), set(st)
    assert sum(s == ("finished", 0) for s in st) > 0.8 * R
    tot = {k: sum(r["counters"][k] for r in res) for k in ("total_scaled_up_nodes", "total_scaled_down_nodes",
                                                              "total_scaled_up_pods", "total_scaled_down_pods")}
    assert all(v > 0 for v in tot.values()), tot
