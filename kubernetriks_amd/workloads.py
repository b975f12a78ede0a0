"""Synthetic workloads for the BASELINE.json configs (data: synthetic; no network, no trace CSVs).

C1  config.yaml + bundled generic example trace, 1 replica            -> c1_scenario()
C2  31-node default cluster (config.yaml:45-68), seed-perturbed        -> c2_scenario()
C3  4,096 Alibaba-like nodes, Alibaba-like pods, integer arrivals      -> c3_scenario()
C4  HPA pod groups + cluster-autoscaler node groups                    -> c4_scenario()
C5  C3-shaped replicas with a scheduler/autoscaler parameter sweep     -> c5_params()

Per-replica variation ("seed-perturbed traces") is applied on the device by the engine's init
kernel (k10s_engine.h: perturb_pod) when k10s_replica_params.perturb = 1: each trace pod's
duration is scaled by k/16 (k in 8..24) and its cpu/ram requests by k/16 (k in 12..20), with k drawn
from splitmix64(seed, pod's workload-trace position).  `perturb_workload` restates that function
bit-exactly so a replica's trace can be materialized for the CPU oracle.

Alibaba-like statistics are the ones the reference's notebook prints
(experiments/alibaba_demo.ipynb cells 1 and 3).
"""
from __future__ import annotations

import math
import random
from typing import List, Optional

from .scenario import (CANodeGroup, DefaultNodeGroup, GenericClusterTrace, GenericWorkloadTrace, Node, Pod,
                       PodGroup, SimulationConfig, UsageModel, WorkloadEvent, scenario_text)

M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def perturb_pod(seed: int, key: int, cpu: int, ram: int, dur: Optional[float]):
    """Bit-exact restatement of k10s_engine.h perturb_pod."""
    u = splitmix64(seed ^ ((0xD1B54A32D192ED03 * (key + 1)) & M64))
    kd = 8 + u % 17
    kc = 12 + (u >> 20) % 9
    kr = 12 + (u >> 40) % 9
    if dur is not None:
        dur = (dur * float(kd)) * 0.0625
    cpu = ((cpu * kc) >> 4) & 0xFFFFFFFF
    ram = ((ram >> 4) * kr) & M64
    return cpu, ram, dur


def perturb_workload(workload: GenericWorkloadTrace, seed: int) -> GenericWorkloadTrace:
    out = GenericWorkloadTrace()
    for pos, e in enumerate(workload.events):
        if e.kind == "create_pod":
            cpu, ram, dur = perturb_pod(seed, pos, e.pod.cpu, e.pod.ram, e.pod.duration)
            out.events.append(WorkloadEvent(e.timestamp, "create_pod",
                                            pod=Pod(e.pod.name, cpu, ram, dur, dict(e.pod.labels))))
        else:
            out.events.append(e)
    return out


# ----------------------------------------------------------------------------------------------
def c1_scenario() -> str:
    """src/config.yaml with the bundled generic trace (generic_{cluster,workload}_trace_example.yaml)."""
    cfg = SimulationConfig()
    c = GenericClusterTrace()
    lab = {"storage_type": "ssd", "proc_type": "intel"}
    c.create_node(1, Node("node_21", 16000, 17179869184, dict(lab)))
    c.remove_node(600, "node_21")
    c.create_node(601, Node("node_22", 16000, 17179869184, dict(lab)))
    w = GenericWorkloadTrace()
    for ts, name, dur in ((550, "pod_16", 21.0), (551, "pod_25", 76.0), (552, "pod_42", 4.0), (553, "pod_101", 4221.0)):
        w.create_pod(ts, Pod(name, 4000, 8589934592, dur))
    w.remove_pod(5001, "pod_42")
    return scenario_text(cfg, c, w)


def default_cluster_31() -> List[DefaultNodeGroup]:
    """The (commented) default cluster of src/config.yaml:45-68."""
    return [DefaultNodeGroup(None, Node("super_node_1024cpu_512gb", 1024000, 549755813888)),
            DefaultNodeGroup(10, Node("default_128cpu_256gb_node", 128000, 274877906944)),
            DefaultNodeGroup(20, Node("default_64cpu_128gb_node", 64000, 137438953472))]


def c2_workload(n_pods: int = 2000, seed: int = 123, horizon: float = 5000.0) -> GenericWorkloadTrace:
    """Pod distribution of tests/test_determinism.rs:49-68 (cpu ceil(U*1000) mcpu, ram U*1e10 B,
    duration U*1000 s), with arrivals over `horizon` seconds."""
    rng = random.Random(seed)
    w = GenericWorkloadTrace()
    for i in range(n_pods):
        w.create_pod(rng.random() * horizon,
                     Pod(f"pod_{i}", int(math.ceil(rng.random() * 1000.0)), int(rng.random() * 10000000000.0),
                         rng.random() * 1000.0))
    return w


def c2_parts(n_pods: int = 2000, seed: int = 123):
    """(config, cluster trace, workload trace) of C2: the 31-node default cluster, no cluster trace."""
    cfg = SimulationConfig()
    cfg.default_cluster = default_cluster_31()
    return cfg, GenericClusterTrace(), c2_workload(n_pods, seed)


def c2_scenario(n_pods: int = 2000, seed: int = 123) -> str:
    return scenario_text(*c2_parts(n_pods, seed))


def c2_survey_parts(n_max: int = 10000, seed: int = 123, horizon: float = 100000.0):
    """C2 at its SURVEY.md §8(d) size: the 31-node default cluster and a master trace of n_max pods
    drawn like tests/test_determinism.rs:49-68 (arrival U*1e5 s, cpu ceil(U*1000) mcpu, ram
    U*1e10 B, duration U*1000 s).  Replica r runs the first ceil(U_r * n_max) of them
    (c2_survey_params: k10s_replica_params.workload_prefix), seed-perturbed."""
    cfg = SimulationConfig()
    cfg.default_cluster = default_cluster_31()
    return cfg, GenericClusterTrace(), c2_workload(n_max, seed, horizon)


def c2_survey_prefix(r: int, n_max: int = 10000, base_seed: int = 123) -> int:
    """Replica r's trace length ceil(U * n_max), U from its own seed (test_determinism.rs:49)."""
    return max(1, int(math.ceil(random.Random(base_seed + r).random() * n_max)))


def c2_survey_params(defaults, n: int, base_seed: int = 123, n_max: int = 10000, replica_offset: int = 0):
    out = replica_params(defaults, n, base_seed=base_seed, perturb=True, replica_offset=replica_offset)
    for i, p in enumerate(out):
        p.workload_prefix = c2_survey_prefix(replica_offset + i, n_max, base_seed)
    return out


# ---- Alibaba-like (C3) ------------------------------------------------------------------------
ALIBABA_NODE_MEM = 0.6899697150104833   # modal machine memory (cluster.rs test fixture / notebook)
GIB128 = 128 * 1024 * 1024 * 1024


def _machine_mem(rng: random.Random) -> float:
    # notebook: 1313 machines, mean 0.692729, sd 0.029690, min 0.574788, quartiles ~0.68997, max 1.0
    r = rng.random()
    if r < 0.85:
        return ALIBABA_NODE_MEM
    if r < 0.93:
        return 0.690001
    if r < 0.97:
        return rng.uniform(0.574788, 0.68997)
    return rng.uniform(0.69, 1.0)


def _task_mem(rng: random.Random) -> float:
    # notebook quantiles of normalized memory request: min 0.003815, 25% 0.004110, 50% 0.007941,
    # 75% 0.009334, max 0.127332
    r = rng.random()
    if r < 0.25:
        return rng.uniform(0.003815, 0.004110)
    if r < 0.5:
        return rng.uniform(0.004110, 0.007941)
    if r < 0.75:
        return rng.uniform(0.007941, 0.009334)
    if r < 0.99:
        return rng.uniform(0.009334, 0.02)
    return rng.uniform(0.02, 0.127332)


def _task_cpu(rng: random.Random) -> int:
    # santicores per instance: mean 49.96, sd 0.946, min 40, quartiles 50, max 60
    r = rng.random()
    c = 50 if r < 0.97 else (40 if r < 0.985 else 60)
    return c * 10  # cpu_santicores * 10 millicores (workload.rs:305-308)


def c3_traces(n_nodes: int = 4096, n_pods: int = 16384, arrival_window: float = 1200.0, seed: int = 2017,
              mean_duration: float = 193.0):
    rng = random.Random(seed)
    c = GenericClusterTrace()
    for k in range(1, n_nodes + 1):
        ram = int(_machine_mem(rng) * float(GIB128))
        c.create_node(0.0, Node(f"alibaba_node_{k}", 64 * 1000, ram))
    w = GenericWorkloadTrace()
    for i in range(n_pods):
        start = float(int(rng.random() * arrival_window) + 1)  # integer seconds: many equal timestamps
        dur = float(max(1, int(rng.expovariate(1.0 / mean_duration))))
        ram = int(_task_mem(rng) * float(GIB128))
        w.create_pod(start, Pod(f"{1000 + i // 64}_{i}_{i}", _task_cpu(rng), ram, dur))
    return c, w


def c3_backlog_traces(n_nodes: int = 4096, n_pods: int = 16384, arrival_window: float = 1200.0, seed: int = 2018,
                      mean_duration: float = 1500.0, ram_frac=(0.3, 0.5)):
    """C3 under load (rho ~ 0.9-1.2 of the RAM-bound capacity, "so backlogs and
    retries occur").  Same 4,096 Alibaba-like nodes; each pod asks for a fraction `ram_frac` of a
    modal node's RAM, so a node holds 2-4 pods, and stays for an exponential duration (mean
    `mean_duration` s, integer seconds).  With 16,384 arrivals over 1,200 s the concurrent demand
    (~ 13.7 pods/s x 1,500 s x (1 - e^-0.8) = 11.3 k pods at t = 1,200 s) exceeds what ~ 4,096
    nodes x 2-3 pods hold, so pods fail attempts (~7 attempts per placement), wait in the
    unschedulable map and are moved back on every pod finish (scheduler.rs:174-244, 289-304,
    422-440); with the conditional move enabled they stay there and the 300-s flush moves them."""
    rng = random.Random(seed)
    c = GenericClusterTrace()
    for k in range(1, n_nodes + 1):
        ram = int(_machine_mem(rng) * float(GIB128))
        c.create_node(0.0, Node(f"alibaba_node_{k}", 64 * 1000, ram))
    node_ram = ALIBABA_NODE_MEM * float(GIB128)
    w = GenericWorkloadTrace()
    for i in range(n_pods):
        start = float(int(rng.random() * arrival_window) + 1)
        dur = float(max(1, int(rng.expovariate(1.0 / mean_duration))))
        ram = int(rng.uniform(ram_frac[0], ram_frac[1]) * node_ram)
        w.create_pod(start, Pod(f"{1000 + i // 64}_{i}_{i}", _task_cpu(rng), ram, dur))
    return c, w


def c3_scenario(n_nodes: int = 4096, n_pods: int = 16384, arrival_window: float = 1200.0, seed: int = 2017) -> str:
    cfg = SimulationConfig()
    c, w = c3_traces(n_nodes, n_pods, arrival_window, seed)
    return scenario_text(cfg, c, w)


# ---- HPA + CA (C4) ----------------------------------------------------------------------------
def c4_scenario(n_batch_pods: int = 400, seed: int = 7) -> str:
    """tests/test_hpa.rs pod group + config.yaml:14-33 CA node groups, with a burst of batch pods
    that forces scale-up and then drains (scale-down)."""
    return scenario_text(*c4_parts(n_batch_pods, seed))


def c4_parts(n_batch_pods: int = 400, seed: int = 7):
    """(config, cluster trace, workload trace) of C4 (see c4_scenario)."""
    rng = random.Random(seed)
    cfg = SimulationConfig()
    cfg.hpa_enabled = True
    cfg.ca_enabled = True
    cfg.ca_max_node_count = 200
    cfg.ca_node_groups = [CANodeGroup("autoscaler_128cpu_256gb_node", 50, 128000, 274877906944),
                          CANodeGroup("autoscaler_64cpu_128gb_node", None, 64000, 137438953472)]
    c = GenericClusterTrace().create_node(5.0, Node("trace_node_42", 64000, 68719476736))
    w = GenericWorkloadTrace()
    g = PodGroup("pod_group_1", 5, 100, Pod("pod_group_1", 100, 104857600, None), 0.6, None,
                 UsageModel("pod_group", units=[(500.0, 8.0), (200.0, 2.0)]), None)
    w.events.append(WorkloadEvent(59.5, "create_pod_group", pod_group=g))
    for i in range(n_batch_pods):
        w.create_pod(float(100 + int(rng.random() * 300)),
                     Pod(f"batch_{i}", rng.choice([4000, 8000, 16000]), rng.choice([8, 16, 32]) << 30,
                         float(rng.randint(60, 600))))
    return cfg, c, w


# ---- C5 with the autoscalers live ------------------------------------------------------------
CA_GROUPS_CONFIG_YAML = (("autoscaler_128cpu_256gb_node", 50, 128000, 274877906944),   # src/config.yaml:14-33
                         ("autoscaler_64cpu_128gb_node", None, 64000, 137438953472))


def c5_autoscaled_parts(n_nodes: int = 4096, n_pods: int = 16384, n_big: Optional[int] = None,
                        arrival_window: float = 1200.0, seed: int = 2019, big_start: float = 300.0,
                        big_window: float = 60.0, big_gap: float = 600.0):
    """(config, cluster trace, workload trace) of the C5 sweep with its autoscaler axes live
    (CA scale-down threshold and HPA tolerance over C3-shaped clusters).

    * cluster: the C3 nodes (Alibaba-like machines, at most 128 GiB of RAM each);
    * config: the cluster autoscaler of src/config.yaml:14-33 enabled (max_node_count 200; node
      groups autoscaler_128cpu_256gb_node, max 50, and autoscaler_64cpu_128gb_node) and the HPA on;
    * workload: n_pods - n_big Alibaba-like pods (c3_traces statistics) over `arrival_window` and
      two bursts of n_big / 2 pods of 16 cores / 180 GiB (135-225 GiB after seed perturbation), over
      [big_start, big_start + big_window] and `big_gap` seconds later.  They fit no trace node, only
      the 256-GiB template: they wait in the unscheduled cache, the CA scales that group up, and the
      Alibaba pods that arrive meanwhile land on the new empty nodes (LeastAllocated); when a burst
      drains, the CA scales those nodes down once their remaining pods can be moved elsewhere
      (scale_down), then up again for the second burst.  Default n_big: 48 per 16,384 pods (within
      the group's max of 50, so a burst does not queue behind itself: under move-all every pod
      finish retries every waiting pod, and a queue of hundreds would turn the run into a retry storm);
    * the test_hpa.rs pod group (tests/test_hpa.rs:28-64), whose load cycle drives the HPA up and down.
    Some parameter cells hit a reference panic: the HPA removes a group pod whose node the CA has
    just scaled down, and the node component unwraps its reclaimed runtime (node_component.rs
    RemovePodRequest).  The engine stops such a replica with K10S_REPLICA_ERROR at the same event,
    exactly like the oracle (about 8 % of the sweep's replicas at 1,500 pods).
    """
    if n_big is None:
        n_big = max(2, round(n_pods * 48 / 16384))
    cfg = SimulationConfig()
    cfg.ca_enabled = True
    cfg.ca_max_node_count = 200
    cfg.ca_node_groups = [CANodeGroup(n, m, c, r) for n, m, c, r in CA_GROUPS_CONFIG_YAML]
    cfg.hpa_enabled = True
    cluster, small = c3_traces(n_nodes, n_pods - n_big, arrival_window, seed)
    rng = random.Random(seed + 1)
    w = GenericWorkloadTrace()
    g = PodGroup("pod_group_1", 5, 100, Pod("pod_group_1", 100, 104857600, None), 0.6, None,
                 UsageModel("pod_group", units=[(500.0, 8.0), (200.0, 2.0)]), None)
    w.events.append(WorkloadEvent(59.5, "create_pod_group", pod_group=g))
    w.events.extend(small.events)
    for i in range(n_big):
        t = float(int(big_start + (big_gap if i % 2 else 0.0) + rng.random() * big_window))
        w.create_pod(t, Pod(f"batch_big_{i}", 16000, 180 << 30, float(rng.randint(200, 600))))
    return cfg, cluster, w


# ---- parameter sweep (C5) ---------------------------------------------------------------------
def c5_params(defaults, n: int, base_seed: int = 123, replica_offset: int = 0):
    """Per-replica k10s_replica_params for the 65,536-replica sweep."""
    from .native import ReplicaParams
    out = []
    for i in range(n):
        r = replica_offset + i
        p = ReplicaParams()
        ctypes_copy(p, defaults)
        p.scheduling_cycle_interval = (1.0, 5.0, 10.0, 30.0)[r % 4]
        p.enable_unscheduled_pods_conditional_move = (r // 4) % 2
        f = (0.5, 1.0, 2.0)[(r // 8) % 3]
        p.sched_to_as_network_delay = defaults.sched_to_as_network_delay * f
        p.ps_to_sched_network_delay = defaults.ps_to_sched_network_delay * f
        p.ca_scale_down_utilization_threshold = (0.3, 0.5, 0.7)[(r // 24) % 3]
        p.hpa_target_threshold_tolerance = (0.05, 0.1, 0.2)[(r // 72) % 3]
        p.seed = base_seed + r
        p.perturb = 1
        out.append(p)
    return out


def config_for_params(cfg: SimulationConfig, p) -> SimulationConfig:
    """The SimulationConfig a replica with k10s_replica_params `p` runs under (the per-replica
    sweep axes mapped back onto config.rs fields), so the CPU oracle can replay that replica."""
    import copy
    c = copy.deepcopy(cfg)
    c.scheduling_cycle_interval = p.scheduling_cycle_interval
    c.enable_unscheduled_pods_conditional_move = bool(p.enable_unscheduled_pods_conditional_move)
    for k in ("as_to_ps", "ps_to_sched", "sched_to_as", "as_to_node", "as_to_ca", "as_to_hpa"):
        setattr(c, f"{k}_network_delay", getattr(p, f"{k}_network_delay"))
    c.ca_scan_interval = p.ca_scan_interval
    c.ca_scale_down_utilization_threshold = p.ca_scale_down_utilization_threshold
    c.hpa_scan_interval = p.hpa_scan_interval
    c.hpa_target_threshold_tolerance = p.hpa_target_threshold_tolerance
    c.score_weight = p.score_weight
    c.score_plugins = p.score_plugins
    c.most_allocated_weight = p.most_allocated_weight
    return c


def replica_scenario(cfg: SimulationConfig, cluster: GenericClusterTrace, workload: GenericWorkloadTrace, p) -> str:
    """Scenario text of one replica as the oracle must see it: its parameters and, when perturbed,
    its seed-perturbed workload (the engine applies both on the device)."""
    w = perturb_workload(workload, p.seed) if p.perturb else workload
    if p.workload_prefix:   # the replica's trace: the first workload_prefix events (generic.rs order)
        w = GenericWorkloadTrace(list(w.events[:p.workload_prefix]))
    return scenario_text(config_for_params(cfg, p), cluster, w)


def ctypes_copy(dst, src):
    import ctypes
    ctypes.memmove(ctypes.addressof(dst), ctypes.addressof(src), ctypes.sizeof(dst))


def replica_params(defaults, n: int, base_seed: int = 123, perturb: bool = True, replica_offset: int = 0):
    """Seed-perturbed replicas with the scenario's config (C2/C3)."""
    from .native import ReplicaParams
    out = []
    for i in range(n):
        p = ReplicaParams()
        ctypes_copy(p, defaults)
        p.seed = base_seed + replica_offset + i
        p.perturb = 1 if perturb else 0
        out.append(p)
    return out
