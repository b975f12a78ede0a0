"""Host-side trace/config readers pinned to the reference's own parse tests and
bundled data files.

* tests/golden/reference_parse_tests.json: inputs and expected values of src/trace/generic.rs:126-272
  and src/trace/alibaba_cluster_trace_v2017/cluster.rs:144-201 (transcribed).
* tests/golden/reference_data/: src/config.yaml and src/data/generic_{cluster,workload}_trace_example.yaml
  as shipped by the reference (data files).
C1 (BASELINE.json configs[0]) is built from those files the way main.rs:26-102 does it — config.yaml
switched to the bundled generic trace, the Alibaba block removed (main.rs:62-65 requires exactly one)
— and must run exactly like the hand-built tests/scenarios.py C1.
"""
import json
import os

import pytest

import oracle_bridge as ob
import parity
import scenarios
from hostcheck_bridge import HostEngine
from kubernetriks_amd.scenario import (DENORMALIZATION_BASE, GenericClusterTrace, GenericWorkloadTrace, Node, Pod,
                                       SimulationConfig, alibaba_cluster_trace_from_csv,
                                       alibaba_workload_trace_from_csv, load_traces, load_yaml,
                                       read_machine_events_from_str, scenario_text)

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DATA = os.path.join(GOLD, "reference_data")
FX = json.load(open(os.path.join(GOLD, "reference_parse_tests.json")))


def _cluster_rows(trace):
    out = []
    for e in trace.events:
        if e.kind == "create_node":
            out.append({"timestamp": e.timestamp, "kind": e.kind, "name": e.node.name, "cpu": e.node.cpu,
                        "ram": e.node.ram, "labels": e.node.labels})
        else:
            out.append({"timestamp": e.timestamp, "kind": e.kind, "name": e.node_name})
    return out


def _workload_rows(trace):
    out = []
    for e in trace.events:
        if e.kind == "create_pod":
            out.append({"timestamp": e.timestamp, "kind": e.kind, "name": e.pod.name, "cpu": e.pod.cpu,
                        "ram": e.pod.ram, "duration": e.pod.duration, "labels": e.pod.labels})
        else:
            out.append({"timestamp": e.timestamp, "kind": e.kind, "name": e.pod_name})
    return out


# ---- generic.rs parse tests ---------------------------------------------------------------------
def test_generic_empty_trace():                     # generic.rs:126-141
    y = FX["generic_empty"]["yaml"]
    assert GenericClusterTrace.from_yaml(y).events == []
    assert GenericWorkloadTrace.from_yaml(y).events == []


def test_generic_cluster_trace():                   # generic.rs:143-205
    got = _cluster_rows(GenericClusterTrace.from_yaml(FX["generic_cluster"]["yaml"]))
    assert got == FX["generic_cluster"]["events"]


def test_generic_workload_trace():                  # generic.rs:207-271
    got = _workload_rows(GenericWorkloadTrace.from_yaml(FX["generic_workload"]["yaml"]))
    assert got == FX["generic_workload"]["events"]


# ---- alibaba cluster.rs parse tests -------------------------------------------------------------
@pytest.mark.parametrize("case", ["machine_events_ok", "machine_events_optional"])
def test_machine_event_rows(case):                  # cluster.rs:144-200
    got = [[m.timestamp, m.machine_id, m.event_type, m.event_detail, m.number_of_cpus, m.normalized_memory,
            m.normalized_disk_space] for m in read_machine_events_from_str(FX[case]["csv"])]
    assert got == FX[case]["rows"]


def test_alibaba_cluster_conversion():
    """convert_to_simulator_events (cluster.rs:54-101) on the reference's add row plus soft/hard
    errors: alibaba_node_{id}, cpus x 1000, memory x 2^37 as u64, one removal per added node."""
    rows = FX["machine_events_optional"]["csv"].splitlines()[1]
    text = "\n".join([rows,
                      "5,924,softerror,machine_fail,0,0,0",
                      "7,924,harderror,,0,0,0",          # already removed: skipped
                      "3,777,softerror,,0,0,0",          # never added: skipped
                      "2,12,add,,32,0.5,0.1"]) + "\n"
    ev = _cluster_rows(alibaba_cluster_trace_from_csv(text))
    assert ev == [
        {"timestamp": 0.0, "kind": "create_node", "name": "alibaba_node_924", "cpu": 64000,
         "ram": int(0.6899697150104833 * float(DENORMALIZATION_BASE)), "labels": {}},
        {"timestamp": 2.0, "kind": "create_node", "name": "alibaba_node_12", "cpu": 32000,
         "ram": DENORMALIZATION_BASE // 2, "labels": {}},
        {"timestamp": 5.0, "kind": "remove_node", "name": "alibaba_node_924"}]
    # the second row of the reference's optional-field test has no memory: `unwrap()` panics
    with pytest.raises(ValueError):
        alibaba_cluster_trace_from_csv(FX["machine_events_optional"]["csv"])
    with pytest.raises(ValueError):
        alibaba_cluster_trace_from_csv("1,3,reboot,,0,0,0\n")


# ---- config.yaml + bundled generic traces -> C1 (main.rs flow) ------------------------------------
def _c1_config_dict():
    d = load_yaml(open(os.path.join(DATA, "config.yaml")).read())
    d["trace_config"] = {"generic_trace": {"workload_trace_path": "generic_workload_trace_example.yaml",
                                           "cluster_trace_path": "generic_cluster_trace_example.yaml"}}
    return d


def test_config_yaml_fields():
    cfg = SimulationConfig.from_yaml(open(os.path.join(DATA, "config.yaml")).read())
    assert cfg.seed == 123 and cfg.scheduling_cycle_interval == 10.0
    assert not cfg.enable_unscheduled_pods_conditional_move
    assert (cfg.as_to_ps_network_delay, cfg.ps_to_sched_network_delay, cfg.sched_to_as_network_delay,
            cfg.as_to_node_network_delay, cfg.as_to_ca_network_delay, cfg.as_to_hpa_network_delay) == \
        (0.050, 0.089, 0.023, 0.152, 0.67, 0.50)
    assert not cfg.ca_enabled and cfg.ca_max_node_count == 200
    assert [(g.name, g.max_count, g.cpu, g.ram) for g in cfg.ca_node_groups] == [
        ("autoscaler_128cpu_256gb_node", 50, 128000, 274877906944),
        ("autoscaler_64cpu_128gb_node", None, 64000, 137438953472)]
    assert not cfg.hpa_enabled and cfg.default_cluster == []
    # config.yaml as shipped names the Alibaba trace only
    assert cfg.trace_config.has_alibaba and not cfg.trace_config.has_generic


def test_load_traces_requires_exactly_one_kind():   # main.rs:62-65
    d = _c1_config_dict()
    d["trace_config"]["alibaba_cluster_trace_v2017"] = {"batch_instance_trace_path": "a", "batch_task_trace_path": "b"}
    with pytest.raises(ValueError):
        load_traces(SimulationConfig.from_dict(d), DATA)
    d["trace_config"] = {}
    with pytest.raises(ValueError):
        load_traces(SimulationConfig.from_dict(d), DATA)


def test_c1_from_reference_files_runs_like_hand_built():
    cfg = SimulationConfig.from_dict(_c1_config_dict())
    cluster, workload = load_traces(cfg, DATA)
    assert _cluster_rows(cluster) == [
        {"timestamp": 1.0, "kind": "create_node", "name": "node_21", "cpu": 16000, "ram": 17179869184,
         "labels": {"storage_type": "ssd", "proc_type": "intel"}},
        {"timestamp": 600.0, "kind": "remove_node", "name": "node_21"},
        {"timestamp": 601.0, "kind": "create_node", "name": "node_22", "cpu": 16000, "ram": 17179869184,
         "labels": {"storage_type": "ssd", "proc_type": "intel"}}]
    assert [r["name"] for r in _workload_rows(workload)] == ["pod_16", "pod_25", "pod_42", "pod_101", "pod_42"]
    text = scenario_text(cfg, cluster, workload)
    hand = scenarios.sc_c1_generic_example()
    # the same scenario except the (disabled) CA block config.yaml also declares (node groups,
    # max_node_count 200): with CA off it sizes nothing (simulator.rs:213-221)
    assert [l for l in text.splitlines() if not l.startswith("ca_")] == \
        [l for l in hand.splitlines() if not l.startswith("ca_")]
    runs = []
    for scn in (text, hand):
        od, e = parity.run_pair(HostEngine, scn)
        assert parity.compare(od, e) == []
        runs.append((e.results()[0], e.event_log(0)))
    assert runs[0] == runs[1]
    c = runs[0][0]["counters"]
    assert c["pods_succeeded"] + c["pods_removed"] == c["terminated_pods"] == 4


def test_load_traces_alibaba_kind(tmp_path):
    """The Alibaba branch of main.rs:66-83: machine events optional, workload from the two CSVs."""
    (tmp_path / "inst.csv").write_text("41562,41618,120,686,299,Terminated,1,1,1.5,0.29,1.0,1.2\n"
                                       "100,160,7,8,1,Terminated,1,1,,,,\n")
    (tmp_path / "task.csv").write_text("10718,12897,120,686,2003,Terminated,50,0.016\n"
                                       "1,2,7,8,1,Terminated,100,0.5\n")
    (tmp_path / "mach.csv").write_text("0,1,add,,64,0.5,0.1\n")
    d = {"scheduling_cycle_interval": 10.0, "as_to_ps_network_delay": 0.05, "ps_to_sched_network_delay": 0.01,
         "sched_to_as_network_delay": 0.02, "as_to_node_network_delay": 0.15, "as_to_ca_network_delay": 0.3,
         "as_to_hpa_network_delay": 0.4,
         "trace_config": {"alibaba_cluster_trace_v2017": {"batch_instance_trace_path": "inst.csv",
                                                          "batch_task_trace_path": "task.csv"}}}
    cluster, workload = load_traces(SimulationConfig.from_dict(d), str(tmp_path))
    assert cluster.events == []
    assert [(e.timestamp, e.pod.name, e.pod.cpu) for e in workload.events] == [(100.0, "7_8_1", 1000),
                                                                               (41562.0, "120_686_0", 500)]
    d["trace_config"]["alibaba_cluster_trace_v2017"]["machine_events_trace_path"] = "mach.csv"
    cluster, _ = load_traces(SimulationConfig.from_dict(d), str(tmp_path))
    assert [(e.node.name, e.node.cpu, e.node.ram) for e in cluster.events] == [("alibaba_node_1", 64000, 1 << 36)]
    # the object path equals the reader functions called directly
    assert workload == alibaba_workload_trace_from_csv((tmp_path / "inst.csv").read_text(),
                                                       (tmp_path / "task.csv").read_text())


def test_only_the_reference_algorithms_resolve():
    """the engine runs the reference's only CA / HPA / usage-model algorithms; an
    enabled autoscaler of another type is refused like resolve_*_impl's panic
    (cluster_autoscaler.rs:219-233, horizontal_pod_autoscaler.rs:171-185)."""
    from kubernetriks_amd.scenario import UsageModel
    d = _c1_config_dict()
    d["cluster_autoscaler"] = {"enabled": True, "autoscaler_type": "kube_cluster_autoscaler", "max_node_count": 5}
    assert SimulationConfig.from_dict(d).ca_enabled
    d["cluster_autoscaler"]["autoscaler_type"] = "my_autoscaler"
    with pytest.raises(ValueError):
        SimulationConfig.from_dict(d)
    d["cluster_autoscaler"]["enabled"] = False        # a disabled one is never resolved
    SimulationConfig.from_dict(d)
    d["horizontal_pod_autoscaler"] = {"enabled": True, "autoscaler_type": "other"}
    with pytest.raises(ValueError):
        SimulationConfig.from_dict(d)
    with pytest.raises(ValueError):
        UsageModel.from_dict({"model_name": "linear", "config": "{}"})
