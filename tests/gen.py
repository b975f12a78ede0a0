"""Randomized scenarios for engine-vs-oracle parity fuzzing.  Inputs only; the oracle supplies
the expected outputs.  Designed to hit the reference's ordering hazards: equal timestamps
(integer arrival seconds), equal scores, zero requests, nodes removed while pods run or while
assignments are in flight, node names re-created, pod removals, conditional moves, CA scale
up/down, HPA pod groups."""
from __future__ import annotations

import random

from kubernetriks_amd.scenario import (CANodeGroup, DefaultNodeGroup, GenericClusterTrace, GenericWorkloadTrace,
                                       Node, Pod, PodGroup, SimulationConfig, UsageModel, WorkloadEvent,
                                       scenario_text, test_simulation_config)


def random_scenario(seed: int, n_pods: int = 60, n_nodes: int = 6, horizon: float = 600.0,
                    ca: bool = False, hpa: bool = False, cond_move=None, removals: bool = True,
                    integer_times: bool = None, same_nodes: bool = None) -> str:
    rng = random.Random(seed)
    cfg = test_simulation_config()
    if rng.random() < 0.3:
        cfg = SimulationConfig()  # the bundled config.yaml delays
    cfg.enable_unscheduled_pods_conditional_move = (rng.random() < 0.3) if cond_move is None else cond_move
    cfg.scheduling_cycle_interval = rng.choice([1.0, 5.0, 10.0, 10.0, 30.0])
    if integer_times is None:
        integer_times = rng.random() < 0.5
    if same_nodes is None:
        same_nodes = rng.random() < 0.4

    def ts(lo=0.0, hi=horizon):
        t = rng.uniform(lo, hi)
        return float(int(t)) if integer_times else t

    cluster = GenericClusterTrace()
    if rng.random() < 0.5:
        cfg.default_cluster = [DefaultNodeGroup(rng.randint(1, 3), Node("", 8000, 16 << 30))]
    names = [f"node_{i}" for i in range(n_nodes)]
    alive = {}
    for nm in names:
        cpu = 8000 if same_nodes else rng.choice([2000, 4000, 8000, 16000])
        ram = (16 << 30) if same_nodes else rng.choice([4 << 30, 8 << 30, 16 << 30, 32 << 30])
        t = ts(0, horizon * 0.3)
        cluster.create_node(t, Node(nm, cpu, ram))
        alive[nm] = t
    if removals:
        for nm in list(alive):
            if rng.random() < 0.25:
                t = ts(alive[nm] + 1, horizon)
                cluster.remove_node(t, nm)
                if rng.random() < 0.5:  # re-create the same name later
                    cluster.create_node(ts(t + 1, horizon * 1.5), Node(nm, 8000, 16 << 30))

    workload = GenericWorkloadTrace()
    pods = []
    for i in range(n_pods):
        r = rng.random()
        if r < 0.03:
            cpu, ram = 0, 0
        elif r < 0.06:
            cpu, ram = 0, rng.randint(1, 1 << 30)
        elif r < 0.1:
            cpu, ram = 40000, 1 << 30  # never fits a single node
        else:
            cpu = rng.choice([100, 250, 500, 1000, 2000, 4000])
            ram = rng.choice([1 << 28, 1 << 29, 1 << 30, 2 << 30, 4 << 30])
        dur = float(rng.randint(1, 400)) if integer_times else rng.uniform(0.5, 400.0)
        name = f"pod_{i}"
        workload.create_pod(ts(), Pod(name, cpu, ram, dur))
        pods.append(name)
    if removals:
        for name in pods:
            if rng.random() < 0.08:
                workload.remove_pod(ts(), name)
        if rng.random() < 0.2:
            workload.remove_pod(ts(), "no_such_pod")

    if ca:
        cfg.ca_enabled = True
        cfg.ca_max_node_count = rng.choice([2, 4, 8])
        cfg.ca_scan_interval = rng.choice([10.0, 30.0])
        cfg.ca_scale_down_utilization_threshold = rng.choice([0.3, 0.5, 0.7])
        cfg.ca_node_groups = [CANodeGroup("ca_big", rng.choice([None, 2]), 16000, 32 << 30),
                              CANodeGroup("ca_small", None, 4000, 8 << 30)]
    if hpa:
        cfg.hpa_enabled = True
        cfg.hpa_scan_interval = rng.choice([30.0, 60.0])
        cfg.hpa_target_threshold_tolerance = rng.choice([0.05, 0.1, 0.2])
        for gi in range(rng.randint(1, 2)):
            units = [(rng.choice([100.0, 300.0, 500.0]), float(rng.randint(1, 10))) for _ in range(rng.randint(1, 3))]
            g = PodGroup(f"group_{gi}", rng.randint(1, 6), rng.randint(6, 20), Pod(f"group_{gi}", 100, 100 << 20, None),
                         rng.choice([0.5, 0.6, 0.8]), rng.choice([None, 0.7]),
                         UsageModel("pod_group", units=units),
                         rng.choice([None, UsageModel("constant", usage=0.5)]))
            workload.events.append(WorkloadEvent(ts(0, horizon * 0.5), "create_pod_group", pod_group=g))
    return scenario_text(cfg, cluster, workload)
