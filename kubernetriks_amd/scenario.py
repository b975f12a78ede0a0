"""Host-side inputs of the kubernetriks hot path: config, traces, and the compiled scenario text.

Mirrors the reference's input layer so a config.yaml / generic trace written for the Rust
simulator drives this engine unchanged:

* ``SimulationConfig``           <- src/config.rs:13-37 (+ CA/HPA blocks with their serde defaults:
                                    cluster_autoscaler.rs:124-161, horizontal_pod_autoscaler.rs:97-129,
                                    kube_cluster_autoscaler.rs:33-53, kube_horizontal_pod_autoscaler.rs:284-302)
* ``GenericClusterTrace`` /
  ``GenericWorkloadTrace``       <- src/trace/generic.rs:34-68 (YAML ``!CreateNode`` style enum tags)
* ``AlibabaClusterTraceV2017`` /
  ``AlibabaWorkloadTraceV2017``  <- src/trace/alibaba_cluster_trace_v2017/{cluster,workload}.rs

Everything is lowered to the line-based scenario text (DESIGN.md §Scenario format) that the C++
engine builder (kubernetriks_amd/csrc/k10s_host.cpp) and the CPU oracle both parse.  Floats are
written with ``repr`` (shortest round-trip), so both sides read bit-identical f64 values.
"""
from __future__ import annotations

import csv
import io
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import yaml

U32_MAX = 0xFFFFFFFF
U64_MAX = 0xFFFFFFFFFFFFFFFF


def _f(x: float) -> str:
    x = float(x)
    if math.isnan(x) or math.isinf(x):
        raise ValueError(f"non-finite value {x!r} in scenario")
    return repr(x)


def _check_name(name: str) -> str:
    if not name or any(c.isspace() for c in name) or "#" in name or "=" in name:
        raise ValueError(f"unsupported object name {name!r} (no whitespace, '#', '=')")
    return name


# --------------------------------------------------------------------------------------------
# YAML with serde-style enum tags (!CreateNode, !PrettyTable, ...)
# --------------------------------------------------------------------------------------------
class _TagLoader(yaml.SafeLoader):
    pass


def _tag_constructor(loader, tag_suffix, node):
    if isinstance(node, yaml.MappingNode):
        value = loader.construct_mapping(node, deep=True)
    elif isinstance(node, yaml.SequenceNode):
        value = loader.construct_sequence(node, deep=True)
    else:
        value = loader.construct_scalar(node)
    return {"__tag__": tag_suffix, "value": value}


_TagLoader.add_multi_constructor("!", _tag_constructor)


def load_yaml(text: str):
    return yaml.load(text, Loader=_TagLoader)


# --------------------------------------------------------------------------------------------
# Objects (core/node.rs, core/pod.rs, autoscalers/horizontal_pod_autoscaler/interface.rs)
# --------------------------------------------------------------------------------------------
@dataclass
class Node:
    name: str
    cpu: int
    ram: int
    labels: Dict[str, str] = field(default_factory=dict)

    @staticmethod
    def from_dict(d: dict) -> "Node":
        md = d.get("metadata") or {}
        cap = (d.get("status") or {})["capacity"]
        return Node(str(md.get("name", "") or ""), int(cap["cpu"]), int(cap["ram"]),
                    {str(k): str(v) for k, v in (md.get("labels") or {}).items()})


@dataclass
class UsageModel:
    """ResourceUsageModelConfig (resource_usage/interface.rs:15-18) parsed eagerly."""
    kind: str                      # "constant" | "pod_group"
    usage: float = 0.0
    units: List[Tuple[float, float]] = field(default_factory=list)

    @staticmethod
    def from_dict(d: Optional[dict]) -> Optional["UsageModel"]:
        if d is None:
            return None
        name, cfg = d["model_name"], d["config"]
        parsed = yaml.safe_load(cfg)
        if name == "constant":
            return UsageModel("constant", usage=float(parsed["usage"]))
        if name == "pod_group":
            return UsageModel("pod_group", units=[(float(u["duration"]), float(u["total_load"])) for u in parsed])
        raise ValueError(f"Unsupported resource usage model: {name!r}")

    def token(self) -> str:
        if self.kind == "constant":
            return "constant:" + _f(self.usage)
        return "pod_group:" + ",".join(f"{_f(d)}/{_f(l)}" for d, l in self.units)


@dataclass
class Pod:
    name: str
    cpu: int
    ram: int
    duration: Optional[float]
    labels: Dict[str, str] = field(default_factory=dict)

    @staticmethod
    def from_dict(d: dict) -> "Pod":
        md = d.get("metadata") or {}
        spec = d["spec"]
        req = spec["resources"]["requests"]
        dur = spec.get("running_duration")
        return Pod(str(md.get("name", "") or ""), int(req["cpu"]), int(req["ram"]),
                   None if dur is None else float(dur),
                   {str(k): str(v) for k, v in (md.get("labels") or {}).items()})


@dataclass
class PodGroup:
    name: str
    initial_pod_count: int
    max_pod_count: int
    template: Pod
    target_cpu: Optional[float]
    target_ram: Optional[float]
    cpu_model: Optional[UsageModel]
    ram_model: Optional[UsageModel]

    @staticmethod
    def from_dict(d: dict) -> "PodGroup":
        tgt = d.get("target_resources_usage") or {}
        rum = d.get("resources_usage_model_config") or {}
        return PodGroup(str(d["name"]), int(d["initial_pod_count"]), int(d["max_pod_count"]),
                        Pod.from_dict(d["pod_template"]),
                        None if tgt.get("cpu_utilization") is None else float(tgt["cpu_utilization"]),
                        None if tgt.get("ram_utilization") is None else float(tgt["ram_utilization"]),
                        UsageModel.from_dict(rum.get("cpu_config")),
                        UsageModel.from_dict(rum.get("ram_config")))


# --------------------------------------------------------------------------------------------
# Config (config.rs)
# --------------------------------------------------------------------------------------------
@dataclass
class CANodeGroup:
    name: str
    max_count: Optional[int]
    cpu: int
    ram: int
    labels: Dict[str, str] = field(default_factory=dict)


@dataclass
class DefaultNodeGroup:
    node_count: Optional[int]
    template: Node


@dataclass
class SimulationConfig:
    scheduling_cycle_interval: float = 10.0
    enable_unscheduled_pods_conditional_move: bool = False
    as_to_ps_network_delay: float = 0.050
    ps_to_sched_network_delay: float = 0.089
    sched_to_as_network_delay: float = 0.023
    as_to_node_network_delay: float = 0.152
    as_to_ca_network_delay: float = 0.67
    as_to_hpa_network_delay: float = 0.50
    seed: int = 123
    sim_name: str = "kubernetriks"
    ca_enabled: bool = False
    ca_scan_interval: float = 10.0
    ca_max_node_count: int = 0
    ca_scale_down_utilization_threshold: float = 0.5
    ca_node_groups: List[CANodeGroup] = field(default_factory=list)
    hpa_enabled: bool = False
    hpa_scan_interval: float = 60.0
    hpa_target_threshold_tolerance: float = 0.1
    default_cluster: List[DefaultNodeGroup] = field(default_factory=list)
    score_weight: float = 1.0  # LeastAllocatedResources weight (kube_scheduler.rs:55)
    # The default profile's score plugins (kube_scheduler.rs:44-61) as bits: 1 LeastAllocatedResources,
    # 2 MostAllocatedResources — an extension: the reference registry (plugin.rs:13-23) has only the
    # first, and its config.yaml has no profile section; `scheduler_score_plugins` below adds one.
    score_plugins: int = 1
    most_allocated_weight: float = 1.0
    trace_config: Optional["TraceConfig"] = None   # config.rs:16, 53-71 (host-side only)

    @staticmethod
    def from_dict(d: dict) -> "SimulationConfig":
        c = SimulationConfig()
        c.sim_name = str(d.get("sim_name", c.sim_name))
        c.seed = int(d.get("seed", c.seed))
        c.scheduling_cycle_interval = float(d["scheduling_cycle_interval"])
        # config.rs:27 has no serde default; the reference's own test helper omits it
        #  — treat missing as false, which is what those tests describe.
        c.enable_unscheduled_pods_conditional_move = bool(d.get("enable_unscheduled_pods_conditional_move", False))
        for k in ("as_to_ps", "ps_to_sched", "sched_to_as", "as_to_node", "as_to_ca", "as_to_hpa"):
            setattr(c, f"{k}_network_delay", float(d[f"{k}_network_delay"]))
        ca = d.get("cluster_autoscaler")
        if ca:
            c.ca_enabled = bool(ca.get("enabled", False))
            # resolve_cluster_autoscaler_impl (cluster_autoscaler.rs:219-233): only the kube algorithm
            if c.ca_enabled and ca.get("autoscaler_type", "kube_cluster_autoscaler") != "kube_cluster_autoscaler":
                raise ValueError("Unsupported cluster autoscaler implementation")
            c.ca_scan_interval = float(ca.get("scan_interval", 10.0))
            c.ca_max_node_count = int(ca.get("max_node_count", 0))
            kca = ca.get("kube_cluster_autoscaler") or {}
            c.ca_scale_down_utilization_threshold = float(kca.get("scale_down_utilization_threshold", 0.5))
            for g in ca.get("node_groups") or []:
                n = Node.from_dict(g["node_template"])
                c.ca_node_groups.append(CANodeGroup(n.name, None if g.get("max_count") is None else int(g["max_count"]),
                                                    n.cpu, n.ram, n.labels))
        hpa = d.get("horizontal_pod_autoscaler")
        if hpa:
            c.hpa_enabled = bool(hpa.get("enabled", False))
            # resolve_horizontal_pod_autoscaler_impl (horizontal_pod_autoscaler.rs:171-185)
            if c.hpa_enabled and hpa.get("autoscaler_type",
                                         "kube_horizontal_pod_autoscaler") != "kube_horizontal_pod_autoscaler":
                raise ValueError("Unsupported horizontal pod autoscaler implementation")
            c.hpa_scan_interval = float(hpa.get("scan_interval", 60.0))
            khpa = hpa.get("kube_horizontal_pod_autoscaler_config") or {}
            c.hpa_target_threshold_tolerance = float(khpa.get("target_threshold_tolerance", 0.1))
        for g in d.get("default_cluster") or []:
            c.default_cluster.append(DefaultNodeGroup(None if g.get("node_count") is None else int(g["node_count"]),
                                                      Node.from_dict(g["node_template"])))
        if d.get("trace_config") is not None:
            c.trace_config = TraceConfig.from_dict(d["trace_config"])
        if d.get("scheduler_score_plugins") is not None:
            c.set_score_plugins(d["scheduler_score_plugins"])
        return c

    SCORE_PLUGIN_BITS = {"LeastAllocatedResources": 1, "MostAllocatedResources": 2}

    def set_score_plugins(self, plugins) -> None:
        """Extension key `scheduler_score_plugins`: a list of {name, weight} like the default profile's
        Plugins.score (kube_scheduler.rs:29-41, 52-55).  Unknown names are refused like
        PLUGIN_REGISTRY.get(..).unwrap() (kube_scheduler.rs:124); a plugin may appear once.  (With
        two plugins the order does not matter: 0.0 + a + b == 0.0 + b + a.)"""
        bits = 0
        for p in plugins:
            name = p["name"]
            if name not in self.SCORE_PLUGIN_BITS:
                raise ValueError(f"unknown score plugin {name!r}")
            b = self.SCORE_PLUGIN_BITS[name]
            if bits & b:
                raise ValueError(f"score plugin {name!r} listed twice")
            bits |= b
            w = float(p["weight"])          # Plugin.weight.unwrap() (kube_scheduler.rs:131)
            if b == 1:
                self.score_weight = w
            else:
                self.most_allocated_weight = w
        if bits == 0:
            raise ValueError("scheduler_score_plugins is empty")
        self.score_plugins = bits

    @staticmethod
    def from_yaml(text: str) -> "SimulationConfig":
        return SimulationConfig.from_dict(load_yaml(text))

    def lines(self) -> List[str]:
        out = [
            f"config scheduling_cycle_interval {_f(self.scheduling_cycle_interval)}",
            f"config enable_unscheduled_pods_conditional_move {int(self.enable_unscheduled_pods_conditional_move)}",
        ]
        for k in ("as_to_ps", "ps_to_sched", "sched_to_as", "as_to_node", "as_to_ca", "as_to_hpa"):
            out.append(f"config {k}_network_delay {_f(getattr(self, k + '_network_delay'))}")
        if self.score_weight != 1.0:
            out.append(f"config score_weight {_f(self.score_weight)}")
        if self.score_plugins != 1:
            out.append(f"config score_plugins {int(self.score_plugins)}")
        if self.most_allocated_weight != 1.0:
            out.append(f"config most_allocated_weight {_f(self.most_allocated_weight)}")
        out.append(f"ca_config enabled {int(self.ca_enabled)} scan_interval {_f(self.ca_scan_interval)} "
                   f"max_node_count {int(self.ca_max_node_count)} scale_down_utilization_threshold "
                   f"{_f(self.ca_scale_down_utilization_threshold)}")
        for g in self.ca_node_groups:
            lab = "".join(f" {_check_name(k)}={_check_name(v)}" for k, v in g.labels.items())
            out.append(f"ca_group {_check_name(g.name)} {'-' if g.max_count is None else int(g.max_count)} "
                       f"{int(g.cpu)} {int(g.ram)}{lab}")
        out.append(f"hpa_config enabled {int(self.hpa_enabled)} scan_interval {_f(self.hpa_scan_interval)} "
                   f"target_threshold_tolerance {_f(self.hpa_target_threshold_tolerance)}")
        for g in self.default_cluster:
            t = g.template
            lab = "".join(f" {_check_name(k)}={_check_name(v)}" for k, v in t.labels.items())
            out.append(f"default_group {'-' if g.node_count is None else int(g.node_count)} "
                       f"{_check_name(t.name) if t.name else '-'} {int(t.cpu)} {int(t.ram)}{lab}")
        return out


@dataclass
class TraceConfig:
    """TraceConfig (config.rs:53-71): exactly one of the two must be set (main.rs:62-65)."""
    generic_cluster_trace_path: Optional[str] = None
    generic_workload_trace_path: Optional[str] = None
    alibaba_batch_instance_trace_path: Optional[str] = None
    alibaba_batch_task_trace_path: Optional[str] = None
    alibaba_machine_events_trace_path: Optional[str] = None
    has_generic: bool = False
    has_alibaba: bool = False

    @staticmethod
    def from_dict(d: dict) -> "TraceConfig":
        t = TraceConfig()
        g = d.get("generic_trace")
        if g is not None:
            t.has_generic = True
            t.generic_cluster_trace_path = str(g["cluster_trace_path"])
            t.generic_workload_trace_path = str(g["workload_trace_path"])
        a = d.get("alibaba_cluster_trace_v2017")
        if a is not None:
            t.has_alibaba = True
            t.alibaba_batch_instance_trace_path = str(a["batch_instance_trace_path"])
            t.alibaba_batch_task_trace_path = str(a["batch_task_trace_path"])
            m = a.get("machine_events_trace_path")
            t.alibaba_machine_events_trace_path = None if m is None else str(m)
        return t


def load_traces(config: SimulationConfig, base_dir: str = ".") -> Tuple["GenericClusterTrace", "GenericWorkloadTrace"]:
    """The trace-selection flow of main.rs:58-95: exactly one trace kind; the Alibaba v2017 kind
    reads batch_instance / batch_task CSVs and, when given, machine events (else an empty cluster
    trace); the generic kind reads the two YAML traces.  Relative paths are taken from base_dir
    (the reference resolves them from its working directory)."""
    import os
    tc = config.trace_config
    if tc is None:
        raise ValueError("config has no trace_config (main.rs:60 unwraps it)")
    if tc.has_alibaba == tc.has_generic:
        raise ValueError("only one of trace config must be set")   # main.rs:62-65

    def rd(p):
        with open(os.path.join(base_dir, p), newline="") as f:
            return f.read()

    if tc.has_alibaba:
        cluster = (alibaba_cluster_trace_from_csv(rd(tc.alibaba_machine_events_trace_path))
                   if tc.alibaba_machine_events_trace_path else GenericClusterTrace())
        return cluster, alibaba_workload_trace_from_csv(rd(tc.alibaba_batch_instance_trace_path),
                                                        rd(tc.alibaba_batch_task_trace_path))
    return (GenericClusterTrace.from_yaml(rd(tc.generic_cluster_trace_path)),
            GenericWorkloadTrace.from_yaml(rd(tc.generic_workload_trace_path)))


def test_simulation_config(**overrides) -> SimulationConfig:
    """default_test_simulation_config (src/test_util/helpers.rs:60-81)."""
    c = SimulationConfig(scheduling_cycle_interval=10.0, as_to_ps_network_delay=0.050,
                         ps_to_sched_network_delay=0.010, sched_to_as_network_delay=0.020,
                         as_to_node_network_delay=0.150, as_to_ca_network_delay=0.30,
                         as_to_hpa_network_delay=0.40, seed=123, sim_name="test_kubernetriks")
    for k, v in overrides.items():
        setattr(c, k, v)
    return c


# --------------------------------------------------------------------------------------------
# Traces (trace/generic.rs, trace/alibaba_cluster_trace_v2017/*.rs)
# --------------------------------------------------------------------------------------------
@dataclass
class ClusterEvent:
    timestamp: float
    kind: str                 # "create_node" | "remove_node"
    node: Optional[Node] = None
    node_name: str = ""


@dataclass
class WorkloadEvent:
    timestamp: float
    kind: str                 # "create_pod" | "remove_pod" | "create_pod_group"
    pod: Optional[Pod] = None
    pod_name: str = ""
    pod_group: Optional[PodGroup] = None


@dataclass
class GenericClusterTrace:
    events: List[ClusterEvent] = field(default_factory=list)

    @staticmethod
    def from_yaml(text: str) -> "GenericClusterTrace":
        d = load_yaml(text) or {}
        out = GenericClusterTrace()
        for e in d.get("events") or []:
            et = e["event_type"]
            tag, v = et["__tag__"], et["value"]
            if tag == "CreateNode":
                out.events.append(ClusterEvent(float(e["timestamp"]), "create_node", node=Node.from_dict(v["node"])))
            elif tag == "RemoveNode":
                out.events.append(ClusterEvent(float(e["timestamp"]), "remove_node", node_name=str(v["node_name"])))
            else:
                raise ValueError(f"unknown cluster event {tag}")
        return out

    def create_node(self, ts: float, node: Node) -> "GenericClusterTrace":
        self.events.append(ClusterEvent(float(ts), "create_node", node=node))
        return self

    def remove_node(self, ts: float, name: str) -> "GenericClusterTrace":
        self.events.append(ClusterEvent(float(ts), "remove_node", node_name=name))
        return self


@dataclass
class GenericWorkloadTrace:
    events: List[WorkloadEvent] = field(default_factory=list)

    @staticmethod
    def from_yaml(text: str) -> "GenericWorkloadTrace":
        d = load_yaml(text) or {}
        out = GenericWorkloadTrace()
        for e in d.get("events") or []:
            et = e["event_type"]
            tag, v = et["__tag__"], et["value"]
            ts = float(e["timestamp"])
            if tag == "CreatePod":
                out.events.append(WorkloadEvent(ts, "create_pod", pod=Pod.from_dict(v["pod"])))
            elif tag == "RemovePod":
                out.events.append(WorkloadEvent(ts, "remove_pod", pod_name=str(v["pod_name"])))
            elif tag == "CreatePodGroup":
                out.events.append(WorkloadEvent(ts, "create_pod_group", pod_group=PodGroup.from_dict(v["pod_group"])))
            else:
                raise ValueError(f"unknown workload event {tag}")
        return out

    def create_pod(self, ts: float, pod: Pod) -> "GenericWorkloadTrace":
        self.events.append(WorkloadEvent(float(ts), "create_pod", pod=pod))
        return self

    def remove_pod(self, ts: float, name: str) -> "GenericWorkloadTrace":
        self.events.append(WorkloadEvent(float(ts), "remove_pod", pod_name=name))
        return self


DENORMALIZATION_BASE = 128 * 1024 * 1024 * 1024   # alibaba .../common.rs:3
CPU_BASE = 1000                                   # alibaba .../common.rs:6


def _f64_as_u64(x: float) -> int:
    """Rust `f64 as u64` (saturating, NaN -> 0)."""
    if math.isnan(x) or x <= 0:
        return 0
    if x >= 18446744073709551616.0:
        return U64_MAX
    return int(x)


def _opt_int(s: str) -> Optional[int]:
    return None if s == "" else int(s)


def _opt_float(s: str) -> Optional[float]:
    return None if s == "" else float(s)


@dataclass
class MachineEvent:
    """One server_event.csv row (cluster.rs:16-38)."""
    timestamp: int
    machine_id: int
    event_type: str
    event_detail: Optional[str]
    number_of_cpus: Optional[int]
    normalized_memory: Optional[float]
    normalized_disk_space: Optional[float]


def read_machine_events_from_str(text: str) -> List[MachineEvent]:
    """read_machine_events_from_str (cluster.rs:106-118): header-less CSV, empty cells -> None."""
    out = []
    for row in csv.reader(io.StringIO(text)):
        if not row:
            continue
        row = row + [""] * (7 - len(row))
        out.append(MachineEvent(int(row[0]), int(row[1]), row[2], row[3] if row[3] != "" else None,
                                _opt_int(row[4]), _opt_float(row[5]), _opt_float(row[6])))
    return out


def alibaba_cluster_trace_from_csv(text: str) -> GenericClusterTrace:
    """AlibabaClusterTraceV2017::convert_to_simulator_events (cluster.rs:54-101): nodes named
    alibaba_node_{machine_id}; a soft/hard error removes a node once, and only one that was
    added; the events are stable-sorted by timestamp."""
    out = GenericClusterTrace()
    created, removed = set(), set()
    for me in read_machine_events_from_str(text):
        ts, mid, etype = me.timestamp, me.machine_id, me.event_type
        name = f"alibaba_node_{mid}"
        if etype == "add":
            created.add(name)
            cpu = me.number_of_cpus
            mem = me.normalized_memory
            if cpu is None or mem is None:
                raise ValueError("add event without cpus/memory (reference unwrap panics)")
            conv_cpu = (cpu * CPU_BASE) & U32_MAX                      # `as u32` truncation
            conv_ram = _f64_as_u64(mem * float(DENORMALIZATION_BASE))
            out.events.append(ClusterEvent(float(ts), "create_node", node=Node(name, conv_cpu, conv_ram)))
        elif etype in ("softerror", "harderror"):
            if name in removed or name not in created:
                continue
            removed.add(name)
            out.events.append(ClusterEvent(float(ts), "remove_node", node_name=name))
        else:
            raise ValueError(f"Unsupported operation for a node in alibaba cluster trace: {etype}")
    out.events.sort(key=lambda e: e.timestamp)   # cluster.rs:99 (stable)
    return out


def alibaba_workload_trace_from_csv(instances_text: str, tasks_text: str) -> GenericWorkloadTrace:
    """AlibabaWorkloadTraceV2017::convert_to_simulator_events (workload.rs:124-141) over
    make_pods_from_instances (56-120): the create_pod events stable-sorted by start time."""
    tasks = {}
    for row in csv.reader(io.StringIO(tasks_text)):
        if not row:
            continue
        tid = int(row[3])
        if tid in tasks:
            raise ValueError(f"duplicated task id: {tid}")
        tasks[tid] = (_opt_int(row[6]), _opt_float(row[7]))
    out = GenericWorkloadTrace()
    pod_no = 0
    for row in csv.reader(io.StringIO(instances_text)):
        if not row:
            continue
        start, end, job, task = _opt_int(row[0]), _opt_int(row[1]), _opt_int(row[2]), _opt_int(row[3])
        if start is None or end is None or task is None or task not in tasks:
            continue
        cpu_sc, mem = tasks[task]
        if cpu_sc is None or mem is None:
            continue
        if start <= 0 or end <= 0 or start >= end:
            continue
        if job is None:   # workload.rs:91 `instance.job_id.unwrap()` panics
            raise ValueError(f"instance of task {task} has no job id")
        name = f"{job}_{task}_{pod_no}"
        pod_no += 1
        pod = Pod(name, (cpu_sc * 10) & U32_MAX, _f64_as_u64(mem * float(DENORMALIZATION_BASE)), float(end - start))
        out.events.append(WorkloadEvent(float(start), "create_pod", pod=pod))
    # convert_to_simulator_events (workload.rs:124-141) returns the events stable-sorted by start
    # time; positions in this list are the engine's perturbation keys, as in the binary block
    out.events.sort(key=lambda e: e.timestamp)
    return out


# --------------------------------------------------------------------------------------------
# Scenario text (DESIGN.md §Scenario format)
# --------------------------------------------------------------------------------------------
def _model_token(m: Optional[UsageModel]) -> str:
    return "none" if m is None else m.token()


def scenario_text(config: SimulationConfig, cluster: GenericClusterTrace, workload: GenericWorkloadTrace) -> str:
    lines = ["k10s_scenario 1"]
    lines += config.lines()
    for e in cluster.events:
        if e.kind == "create_node":
            n = e.node
            lab = "".join(f" {_check_name(k)}={_check_name(v)}" for k, v in n.labels.items())
            lines.append(f"cluster {_f(e.timestamp)} create_node {_check_name(n.name)} {int(n.cpu)} {int(n.ram)}{lab}")
        else:
            lines.append(f"cluster {_f(e.timestamp)} remove_node {_check_name(e.node_name)}")
    for e in workload.events:
        if e.kind == "create_pod":
            p = e.pod
            lab = "".join(f" {_check_name(k)}={_check_name(v)}" for k, v in p.labels.items())
            dur = "none" if p.duration is None else _f(p.duration)
            lines.append(f"workload {_f(e.timestamp)} create_pod {_check_name(p.name)} {int(p.cpu)} {int(p.ram)} {dur}{lab}")
        elif e.kind == "remove_pod":
            lines.append(f"workload {_f(e.timestamp)} remove_pod {_check_name(e.pod_name)}")
        else:
            g = e.pod_group
            t = g.template
            dur = "none" if t.duration is None else _f(t.duration)
            tc = "-" if g.target_cpu is None else _f(g.target_cpu)
            tr = "-" if g.target_ram is None else _f(g.target_ram)
            lines.append(f"workload {_f(e.timestamp)} create_pod_group {_check_name(g.name)} {int(g.initial_pod_count)} "
                         f"{int(g.max_pod_count)} {int(t.cpu)} {int(t.ram)} {dur} {tc} {tr} "
                         f"{_model_token(g.cpu_model)} {_model_token(g.ram_model)}")
    lines.append("end")
    return "\n".join(lines) + "\n"


def pods_blob(pods: Sequence[Tuple[float, "Pod"]]) -> bytes:
    """Binary SoA block of create_pod events for k10s_engine_create_bulk (include/k10s.h): ts f64,
    cpu u32, ram u64, duration f64 (NaN = long-running), names as one offset table + bytes.  Pods
    with labels must go through the text format."""
    import numpy as np
    n = len(pods)
    ts = np.array([float(t) for t, _ in pods], dtype="<f8")
    cpu = np.array([int(p.cpu) for _, p in pods], dtype="<u4")
    ram = np.array([int(p.ram) for _, p in pods], dtype="<u8")
    dur = np.array([math.nan if p.duration is None else float(p.duration) for _, p in pods], dtype="<f8")
    names = [_check_name(p.name).encode() for _, p in pods]
    if any(p.labels for _, p in pods):
        raise ValueError("pods with labels are not supported in the bulk blob")
    off = np.zeros(n + 1, dtype="<u4")
    off[1:] = np.cumsum([len(b) for b in names], dtype=np.uint64)
    pad = b"\0" * (4 * (n & 1))
    return (b"K10SPOD1" + np.array([n], dtype="<u8").tobytes() + ts.tobytes() + cpu.tobytes() + pad +
            ram.tobytes() + dur.tobytes() + off.tobytes() + b"".join(names))


def nodes_blob(events: Sequence["ClusterEvent"]) -> bytes:
    """Binary SoA block of cluster events (create_node / remove_node) for k10s_engine_create_bulk
    (include/k10s.h "K10SNOD1"): ts f64, cpu u32, ram u64, op u32 (0 create, 1 remove), names as
    one offset table + bytes.  Nodes with labels must go through the text format."""
    import numpy as np
    n = len(events)
    ts = np.array([float(e.timestamp) for e in events], dtype="<f8")
    cpu = np.array([int(e.node.cpu) if e.kind == "create_node" else 0 for e in events], dtype="<u4")
    ram = np.array([int(e.node.ram) if e.kind == "create_node" else 0 for e in events], dtype="<u8")
    op = np.array([0 if e.kind == "create_node" else 1 for e in events], dtype="<u4")
    names = [_check_name(e.node.name if e.kind == "create_node" else e.node_name).encode() for e in events]
    if any(e.kind == "create_node" and e.node.labels for e in events):
        raise ValueError("nodes with labels are not supported in the bulk blob")
    off = np.zeros(n + 1, dtype="<u4")
    off[1:] = np.cumsum([len(b) for b in names], dtype=np.uint64)
    pad = b"\0" * (4 * (n & 1))
    return (b"K10SNOD1" + np.array([n], dtype="<u8").tobytes() + ts.tobytes() + cpu.tobytes() + pad +
            ram.tobytes() + op.tobytes() + pad + off.tobytes() + b"".join(names))


def scenario_bulk(config: SimulationConfig, cluster: GenericClusterTrace,
                  workload: GenericWorkloadTrace, cluster_blob: bool = False) -> Tuple[str, bytes]:
    """(scenario text, blob) for k10s_engine_create_bulk: the workload's create_pod events go into a
    binary K10SPOD1 block, and with cluster_blob=True the cluster trace into a K10SNOD1 block;
    everything else stays text.  The engine appends each block after the text's lines of its
    trace, so the result equals scenario_text(...) when the blocked events come last in their
    trace (e.g. a pure pod trace, a whole cluster trace)."""
    pods = [(e.timestamp, e.pod) for e in workload.events if e.kind == "create_pod"]
    rest = GenericWorkloadTrace([e for e in workload.events if e.kind != "create_pod"])
    if cluster_blob:
        return scenario_text(config, GenericClusterTrace(), rest), nodes_blob(cluster.events) + pods_blob(pods)
    return scenario_text(config, cluster, rest), pods_blob(pods)
