"""Scenario builders for the reference's own test cases (inputs only; expected values live in
tests/golden/reference_goldens.json).  Each builder cites the reference test it restates.
"""
from __future__ import annotations

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from kubernetriks_amd.scenario import (DefaultNodeGroup, GenericClusterTrace,  # noqa: E402
                                       GenericWorkloadTrace, Node, Pod, PodGroup, SimulationConfig,
                                       UsageModel, WorkloadEvent, scenario_text,
                                       test_simulation_config)


def pods_cluster_trace() -> GenericClusterTrace:
    """tests/test_pods.rs:16-33 — trace_node_42 (2000 mcpu, 4 GiB) at t=30."""
    return GenericClusterTrace().create_node(30, Node("trace_node_42", 2000, 4294967296))


def pods_workload_trace() -> GenericWorkloadTrace:
    """tests/test_pods.rs:35-72 — pod_0 @41, pod_1 @42 (333 mcpu, 4967296 B, 100 s)."""
    w = GenericWorkloadTrace()
    w.create_pod(41, Pod("pod_0", 333, 4967296, 100.0))
    w.create_pod(42, Pod("pod_1", 333, 4967296, 100.0))
    return w


def sc_pod_arrived_before_node() -> str:                       # test_pods.rs:74-115
    w = GenericWorkloadTrace().create_pod(5, Pod("pod_16", 2000, 4294967296, 100.0))
    return scenario_text(test_simulation_config(), pods_cluster_trace(), w)


def sc_many_pods_one_at_a_time() -> str:                        # test_pods.rs:117-218
    w = GenericWorkloadTrace()
    for i in range(4):
        w.create_pod(40 + i, Pod(f"pod_{i}", 2000, 4294967296, 100.0))
    return scenario_text(test_simulation_config(), pods_cluster_trace(), w)


def sc_node_fits_all_pods() -> str:                             # test_pods.rs:220-313
    w = GenericWorkloadTrace()
    for i, d in enumerate((100.0, 50.0, 25.0)):
        w.create_pod(41 + i, Pod(f"pod_{i}", 333, 294967296, d))
    return scenario_text(test_simulation_config(), pods_cluster_trace(), w)


def sc_node_remove_while_running() -> str:                      # test_pods.rs:315-365
    c = pods_cluster_trace()
    c.remove_node(60.0, "trace_node_42")
    c.create_node(1100.0, Node("trace_node_42", 2000, 4294967296))
    return scenario_text(test_simulation_config(), c, pods_workload_trace())


def sc_node_removed_same_time_as_assignment() -> str:           # test_pods.rs:367-398
    c = pods_cluster_trace()
    c.remove_node(50.0, "trace_node_42")
    return scenario_text(test_simulation_config(), c, pods_workload_trace())


def sc_pod_removals() -> str:                                   # test_pods.rs:400-449
    w = pods_workload_trace()
    w.remove_pod(71.0, "pod_1")
    return scenario_text(test_simulation_config(), pods_cluster_trace(), w)


def sc_pod_removal_concurrent_with_node_removal() -> str:       # test_pods.rs:451-510
    c = pods_cluster_trace()
    w = pods_workload_trace()
    w.remove_pod(70.9, "pod_0")
    c.remove_node(71.0, "trace_node_42")
    w.remove_pod(71.0001, "pod_1")
    c.create_node(500.0, Node("trace_node_42", 2000, 4294967296))
    return scenario_text(test_simulation_config(), c, w)


def sc_removed_pod_frees_place() -> str:                        # test_pods.rs:512-594
    w = GenericWorkloadTrace()
    w.create_pod(40.0, Pod("pod_0", 2000, 4294967296, 200.0))
    w.create_pod(41.0, Pod("pod_1", 2000, 4294967296, 200.0))
    w.remove_pod(120.0, "pod_0")
    return scenario_text(test_simulation_config(), pods_cluster_trace(), w)


def sc_pod_removed_after_finished() -> str:                     # test_pods.rs:596-637
    w = pods_workload_trace()
    w.remove_pod(150.2, "pod_0")
    return scenario_text(test_simulation_config(), pods_cluster_trace(), w)


def sc_hpa() -> str:                                            # tests/test_hpa.rs:10-89
    cfg = test_simulation_config(hpa_enabled=True)
    c = GenericClusterTrace().create_node(5.0, Node("trace_node_42", 64000, 68719476736))
    g = PodGroup("pod_group_1", 5, 100, Pod("pod_group_1", 100, 104857600, None), 0.6, None,
                 UsageModel("pod_group", units=[(500.0, 8.0), (200.0, 2.0)]), None)
    w = GenericWorkloadTrace()
    w.events.append(WorkloadEvent(59.5, "create_pod_group", pod_group=g))
    return scenario_text(cfg, c, w)


def sc_node_creation() -> str:                                  # tests/test_node_creation.rs:15-56
    cfg = test_simulation_config()
    cfg.default_cluster = [DefaultNodeGroup(1, Node("my_node_1", 16000, 8589934592))]
    c = GenericClusterTrace().create_node(30, Node("trace_node_25", 16000, 17179869184))
    return scenario_text(cfg, c, GenericWorkloadTrace())


def sc_default_cluster_no_prefix() -> str:                      # tests/test_default_cluster.rs:25-69
    cfg = test_simulation_config()
    cfg.default_cluster = [
        DefaultNodeGroup(10, Node("", 18000, 18589934592, {"storage_type": "ssd", "proc_type": "intel"})),
        DefaultNodeGroup(20, Node("", 24000, 18589934592)),
    ]
    return scenario_text(cfg, GenericClusterTrace(), GenericWorkloadTrace())


def sc_default_cluster_no_count() -> str:                       # tests/test_default_cluster.rs:71-117
    cfg = test_simulation_config()
    cfg.default_cluster = [
        DefaultNodeGroup(None, Node("", 24000, 18589934592)),
        DefaultNodeGroup(None, Node("", 12000, 10589934592)),
        DefaultNodeGroup(1, Node("", 6000, 185899345)),
        DefaultNodeGroup(1, Node("", 8000, 185899345)),
    ]
    return scenario_text(cfg, GenericClusterTrace(), GenericWorkloadTrace())


def sc_default_cluster_prefix() -> str:                         # tests/test_default_cluster.rs:119-165
    cfg = test_simulation_config()
    cfg.default_cluster = [
        DefaultNodeGroup(2, Node("node_group_1", 32000, 18589934592)),
        DefaultNodeGroup(1, Node("exact_node_name", 6000, 185899345)),
        DefaultNodeGroup(None, Node("exact_node_name_2", 4000, 185899345)),
    ]
    return scenario_text(cfg, GenericClusterTrace(), GenericWorkloadTrace())


def sc_c1_generic_example() -> str:
    """Config C1: src/config.yaml switched to the bundled generic trace
    (src/data/generic_cluster_trace_example.yaml, generic_workload_trace_example.yaml)."""
    cfg = SimulationConfig()  # config.yaml:68-76 delays, cycle 10, conditional move false
    c = GenericClusterTrace()
    c.create_node(1, Node("node_21", 16000, 17179869184, {"storage_type": "ssd", "proc_type": "intel"}))
    c.remove_node(600, "node_21")
    c.create_node(601, Node("node_22", 16000, 17179869184, {"storage_type": "ssd", "proc_type": "intel"}))
    w = GenericWorkloadTrace()
    for ts, name, dur in ((550, "pod_16", 21.0), (551, "pod_25", 76.0), (552, "pod_42", 4.0), (553, "pod_101", 4221.0)):
        w.create_pod(ts, Pod(name, 4000, 8589934592, dur))
    w.remove_pod(5001, "pod_42")
    return scenario_text(cfg, c, w)


ALL_TEST_SCENARIOS = {
    "pod_arrived_before_node": sc_pod_arrived_before_node,
    "many_pods_one_at_a_time": sc_many_pods_one_at_a_time,
    "node_fits_all_pods": sc_node_fits_all_pods,
    "node_remove_while_running": sc_node_remove_while_running,
    "node_removed_same_time_as_assignment": sc_node_removed_same_time_as_assignment,
    "pod_removals": sc_pod_removals,
    "pod_removal_concurrent_with_node_removal": sc_pod_removal_concurrent_with_node_removal,
    "removed_pod_frees_place": sc_removed_pod_frees_place,
    "pod_removed_after_finished": sc_pod_removed_after_finished,
    "hpa": sc_hpa,
    "node_creation": sc_node_creation,
    "default_cluster_no_prefix": sc_default_cluster_no_prefix,
    "default_cluster_no_count": sc_default_cluster_no_count,
    "default_cluster_prefix": sc_default_cluster_prefix,
    "c1_generic_example": sc_c1_generic_example,
}
