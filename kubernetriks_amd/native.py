"""ctypes binding of the engine's C ABI (include/k10s.h) — the Python mirror of the reference's
KubernetriksSimulation surface for the batched-ensemble engine.

The shared library is built in-tree (``build/libk10s.so``, see ``kubernetriks_amd/build.py``).
There is no CPU fallback: without the library or without a GPU every entry point raises.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Optional, Sequence

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("K10S_LIB") or os.path.join(REPO, "build", "libk10s.so")
if not os.path.isabs(LIB_PATH):   # a variant library named relative to the repository (tools/gpu.sh env: steps)
    LIB_PATH = os.path.join(REPO, LIB_PATH)

NUM_COUNTERS = 19
COUNTER_NAMES = [
    "total_nodes_in_trace", "total_pods_in_trace", "pods_succeeded", "pods_unschedulable", "pods_failed",
    "pods_removed", "total_scaled_up_nodes", "total_scaled_down_nodes", "total_scaled_up_pods",
    "total_scaled_down_pods", "processed_nodes", "terminated_pods", "placements", "attempts", "events",
    "nodes_scanned", "nodes_read", "requeued", "flushed",
]
EST_NAMES = ["pod_duration", "pod_schedule_time", "pod_queue_time"]


def _event_kind_names():
    """{kind id: name} from include/k10s_events.h (K10S_EV_AS_CREATE_POD_REQ = 4 -> "AS_CREATE_POD_REQ")."""
    import re
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "k10s_events.h")
    try:
        text = open(path).read()
    except OSError:
        return {}
    return {int(v): k for k, v in re.findall(r"K10S_EV_([A-Z0-9_]+)\s*=\s*(\d+)", text) if k != "NUM_KINDS"}


EVENT_KIND_NAMES = _event_kind_names()

RUN_UNTIL_ALL_FINISHED = 0
RUN_UNTIL_TIME = 1

STATUS = {0: "running", 1: "finished", 2: "error", 3: "time_limit", 4: "stalled"}
K10S_PANIC_MISSING_POD = 4
K10S_PANIC_NEGATIVE_DELAY = 15   # dslab-core add_event refuses an event in the past (include/k10s.h)


HIST_BINS = 32  # K10S_HIST_BINS (include/k10s.h): log2 bins, 0: < 2^-10 s, k: [2^(k-11), 2^(k-10)), 31: >= 2^20 s


class Estimator(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("min", ctypes.c_double), ("max", ctypes.c_double),
                ("mean", ctypes.c_double), ("sum2", ctypes.c_double), ("hist", ctypes.c_uint32 * HIST_BINS)]


class ReplicaResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint32), ("error_code", ctypes.c_uint32), ("error_kind", ctypes.c_uint32),
                ("error_seq", ctypes.c_uint32), ("error_time", ctypes.c_double), ("clock", ctypes.c_double),
                ("counters", ctypes.c_uint64 * NUM_COUNTERS), ("est", Estimator * 3),
                ("unschedulable_len", ctypes.c_uint32), ("active_len", ctypes.c_uint32),
                ("node_count_as", ctypes.c_uint32), ("node_count_ps", ctypes.c_uint32),
                ("node_count_s", ctypes.c_uint32), ("log_len", ctypes.c_uint32),
                ("placements_len", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class ReplicaParams(ctypes.Structure):
    _fields_ = [("scheduling_cycle_interval", ctypes.c_double),
                ("as_to_ps_network_delay", ctypes.c_double), ("ps_to_sched_network_delay", ctypes.c_double),
                ("sched_to_as_network_delay", ctypes.c_double), ("as_to_node_network_delay", ctypes.c_double),
                ("as_to_ca_network_delay", ctypes.c_double), ("as_to_hpa_network_delay", ctypes.c_double),
                ("ca_scan_interval", ctypes.c_double), ("ca_scale_down_utilization_threshold", ctypes.c_double),
                ("hpa_scan_interval", ctypes.c_double), ("hpa_target_threshold_tolerance", ctypes.c_double),
                ("score_weight", ctypes.c_double),
                ("enable_unscheduled_pods_conditional_move", ctypes.c_uint32), ("perturb", ctypes.c_uint32),
                ("seed", ctypes.c_uint64), ("ca_max_node_count", ctypes.c_uint64),
                ("most_allocated_weight", ctypes.c_double), ("score_plugins", ctypes.c_uint32),
                ("workload_prefix", ctypes.c_uint32)]


SCORE_LEAST_ALLOCATED = 1   # k10s_replica_params.score_plugins bits (include/k10s.h)
SCORE_MOST_ALLOCATED = 2


class Capacities(ctypes.Structure):
    _fields_ = [("event_heap", ctypes.c_uint32), ("active_queue", ctypes.c_uint32),
                ("unschedulable", ctypes.c_uint32), ("group_name_bound", ctypes.c_uint32),
                ("ca_name_bound", ctypes.c_uint32), ("event_log", ctypes.c_uint32),
                ("placement_log", ctypes.c_uint32), ("pod_records", ctypes.c_uint32),
                ("delay_fifo", ctypes.c_uint32), ("pruned_scan", ctypes.c_uint32), ("gauge_log", ctypes.c_uint32),
                ("stall_guard", ctypes.c_uint32), ("node_cache", ctypes.c_uint32)]


class GaugeRow(ctypes.Structure):  # k10s_gauge_row (collector.rs:392-407 CSV columns)
    _fields_ = [("time", ctypes.c_double), ("current_nodes", ctypes.c_uint64), ("current_pods", ctypes.c_uint64),
                ("pods_in_scheduling_queues", ctypes.c_uint64), ("node_average_cpu_utilization", ctypes.c_double),
                ("node_average_ram_utilization", ctypes.c_double), ("cluster_total_cpu_utilization", ctypes.c_double),
                ("cluster_total_ram_utilization", ctypes.c_double)]


class LogEntry(ctypes.Structure):
    _fields_ = [("time", ctypes.c_double), ("seq", ctypes.c_uint32), ("kind", ctypes.c_uint16),
                ("slot", ctypes.c_int16), ("pod", ctypes.c_int32), ("node", ctypes.c_int32)]


class Placement(ctypes.Structure):
    _fields_ = [("assign_time", ctypes.c_double), ("pod", ctypes.c_int32), ("node", ctypes.c_int32)]


class PodRecord(ctypes.Structure):
    _fields_ = [("t_running", ctypes.c_double), ("t_finished", ctypes.c_double), ("t_removed", ctypes.c_double),
                ("state", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


def result_to_dict(r: ReplicaResult) -> dict:
    return {
        "status": STATUS.get(r.status, r.status), "error_code": r.error_code, "error_kind": r.error_kind,
        "error_seq": r.error_seq, "error_time": r.error_time, "time": r.clock,
        "counters": {COUNTER_NAMES[i]: int(r.counters[i]) for i in range(NUM_COUNTERS)},
        "estimators": {EST_NAMES[i]: [int(r.est[i].n), r.est[i].min, r.est[i].max, r.est[i].mean,
                                      (r.est[i].sum2 / r.est[i].n) if r.est[i].n else math.nan,
                                      list(r.est[i].hist)]
                       for i in range(3)},
        "unschedulable_len": r.unschedulable_len, "active_len": r.active_len,
        "node_counts": [r.node_count_as, r.node_count_ps, r.node_count_s],
        "log_len": r.log_len, "placements_len": r.placements_len, "flags": r.flags,
    }


def _decl(L, prefix: str):
    """Declare the engine-surface signatures shared by the product library and the test build."""
    vp, u32, u64, i32, dbl = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_double
    P = ctypes.POINTER
    sig = {
        "results": (i32, [vp, P(ReplicaResult)]),
        "event_log": (i32, [vp, u32, P(LogEntry), u32, P(u32)]),
        "placements": (i32, [vp, u32, P(Placement), u32, P(u32)]),
        "gauges": (i32, [vp, u32, P(GaugeRow), u32, P(u32)]),
        "pod_records": (i32, [vp, u32, P(PodRecord), u32, P(u32)]),
        "group_sizes": (i32, [vp, u32, P(u32), P(u32), u32, P(u32)]),
        "num_nodes": (u32, [vp]), "num_pods": (u32, [vp]), "num_groups": (u32, [vp]),
        "node_name": (ctypes.c_char_p, [vp, u32]), "pod_name": (ctypes.c_char_p, [vp, u32]),
        "group_name": (ctypes.c_char_p, [vp, u32]), "replica_bytes": (u64, [vp]),
        "node_entry_bytes": (u32, [vp]),
        "default_params": (i32, [vp, P(ReplicaParams)]),
        "name_bounds": (i32, [vp, P(u32), P(u32)]),
        "capacities": (i32, [vp, P(Capacities), P(u32)]),
        "check_fronts": (i32, [vp, u32, P(ctypes.c_int32)]),
    }
    out = {}
    for name, (res, args) in sig.items():
        if name in ("node_entry_bytes", "name_bounds", "capacities", "check_fronts") and not hasattr(L, prefix + name):
            continue   # a library from an earlier round (A/B tooling)
        f = getattr(L, prefix + name)
        f.restype = res
        f.argtypes = args
        out[name] = f
    return out


class EngineBase:
    """Common result accessors (names resolved through the compiled scenario's rank tables)."""

    _fn: dict
    _h: int
    n_replicas: int

    def _names(self):
        if not hasattr(self, "_node_names"):
            f = self._fn
            self._node_names = [f["node_name"](self._h, i).decode() for i in range(f["num_nodes"](self._h))]
            self._pod_names = [f["pod_name"](self._h, i).decode() for i in range(f["num_pods"](self._h))]
            self._group_names = [f["group_name"](self._h, i).decode() for i in range(f["num_groups"](self._h))]
        return self._node_names, self._pod_names, self._group_names

    def _forget_names(self):
        """A run may regrow the batch's generated-name universes (k10s_engine_name_bounds): the
        name tables are re-read after every run."""
        for a in ("_node_names", "_pod_names", "_group_names"):
            self.__dict__.pop(a, None)

    @property
    def name_bounds(self):
        """(names per pod group, names per CA node group) of the compiled batch; a run that would
        exceed one recompiles the batch with it doubled (include/k10s.h k10s_engine_name_bounds)."""
        g, c = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self._fn["name_bounds"](self._h, ctypes.byref(g), ctypes.byref(c)))
        return int(g.value), int(c.value)

    @property
    def capacities(self):
        """(effective capacities as a dict, regrows since create): event_heap, active_queue,
        unschedulable, the name bounds and delay_fifo as compiled, after any regrow
        (include/k10s.h k10s_engine_capacities)."""
        c, n = Capacities(), ctypes.c_uint32()
        self._check(self._fn["capacities"](self._h, ctypes.byref(c), ctypes.byref(n)))
        return {f: int(getattr(c, f)) for f, _ in Capacities._fields_}, int(n.value)

    def check_fronts(self, r: int = 0) -> int:
        """Test support (include/k10s.h k10s_engine_check_fronts): blocks of replica r whose front
        slots were checked against the node cache; raises if one is wrong; 0 without fronts."""
        out = ctypes.c_int32()
        self._check(self._fn["check_fronts"](self._h, r, ctypes.byref(out)))
        if out.value < 0:
            raise AssertionError(f"replica {r}: block {-out.value - 1} does not hold its front")
        return int(out.value)

    @property
    def node_names(self) -> List[str]:
        return self._names()[0]

    @property
    def pod_names(self) -> List[str]:
        return self._names()[1]

    @property
    def group_names(self) -> List[str]:
        return self._names()[2]

    def default_params(self) -> ReplicaParams:
        p = ReplicaParams()
        self._check(self._fn["default_params"](self._h, ctypes.byref(p)))
        return p

    def raw_results(self):
        arr = (ReplicaResult * self.n_replicas)()
        self._check(self._fn["results"](self._h, arr))
        return arr

    def counter_matrix(self, arr=None):
        """The replicas' counters as one (R, NUM_COUNTERS) uint64 numpy view of a results array
        (no per-replica Python loop)."""
        import numpy as np
        if arr is None:
            arr = self.raw_results()
        return np.ndarray((len(arr), NUM_COUNTERS), dtype="<u8", buffer=arr, offset=ReplicaResult.counters.offset,
                          strides=(ctypes.sizeof(ReplicaResult), 8))

    def results(self) -> List[dict]:
        return [result_to_dict(r) for r in self.raw_results()]

    def event_log(self, r: int, cap: int = 1 << 22) -> List[tuple]:
        buf = (LogEntry * cap)()
        n = ctypes.c_uint32()
        self._check(self._fn["event_log"](self._h, r, buf, cap, ctypes.byref(n)))
        nn, pn, _ = self._names()
        return [(e.seq, e.time, e.kind, pn[e.pod] if e.pod >= 0 else "", nn[e.node] if e.node >= 0 else "", e.slot)
                for e in buf[: n.value]]

    def gauges(self, r: int, cap: int = 1 << 20) -> List[tuple]:
        """Gauge recorder rows (time, current_nodes, current_pods, pods_in_scheduling_queues,
        node_average_cpu, node_average_ram, cluster_total_cpu, cluster_total_ram)."""
        buf = (GaugeRow * cap)()
        n = ctypes.c_uint32()
        self._check(self._fn["gauges"](self._h, r, buf, cap, ctypes.byref(n)))
        return [tuple(getattr(g, f) for f, _ in GaugeRow._fields_) for g in buf[: n.value]]

    def placements(self, r: int, cap: int = 1 << 22) -> List[tuple]:
        buf = (Placement * cap)()
        n = ctypes.c_uint32()
        self._check(self._fn["placements"](self._h, r, buf, cap, ctypes.byref(n)))
        nn, pn, _ = self._names()
        return [(pn[x.pod], nn[x.node], x.assign_time) for x in buf[: n.value]]

    def pod_records(self, r: int) -> Dict[str, tuple]:
        cap = self._fn["num_pods"](self._h)
        buf = (PodRecord * max(cap, 1))()
        n = ctypes.c_uint32()
        self._check(self._fn["pod_records"](self._h, r, buf, cap, ctypes.byref(n)))
        _, pn, _ = self._names()
        return {pn[i]: (buf[i].t_running, buf[i].t_finished, buf[i].t_removed, buf[i].state)
                for i in range(n.value) if buf[i].state != 0}

    def group_sizes(self, r: int) -> Dict[str, tuple]:
        G = self._fn["num_groups"](self._h)
        c = (ctypes.c_uint32 * max(G, 1))()
        t = (ctypes.c_uint32 * max(G, 1))()
        n = ctypes.c_uint32()
        self._check(self._fn["group_sizes"](self._h, r, c, t, G, ctypes.byref(n)))
        _, _, gn = self._names()
        return {gn[i]: (c[i], t[i]) for i in range(n.value)}

    def step_for_duration(self, duration: float, max_events_per_launch: int = 0):
        """KubernetriksSimulation::step_for_duration (simulator.rs:394-396) = dslab
        step_until_time(time() + duration).  Every replica must be at the same clock (as after a
        step_until_time); replicas run to completion have their own clocks and are rejected."""
        clocks = {r.clock for r in self.raw_results()}
        if len(clocks) != 1:
            raise ValueError("step_for_duration needs every replica at the same clock")
        return self.step_until_time(clocks.pop() + duration, max_events_per_launch)

    @property
    def replica_bytes(self) -> int:
        return int(self._fn["replica_bytes"](self._h))

    @property
    def node_entry_bytes(self) -> int:
        """Bytes per node of the node cache each scheduling attempt reads: 8 packed, 12 wide
        (k10s_capacities.node_cache)."""
        f = self._fn.get("node_entry_bytes")
        return int(f(self._h)) if f else 12

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f"engine call failed with {rc}: {self._last_error()}")

    def _last_error(self) -> str:
        return ""


_lib = None


def lib():
    """Load build/libk10s.so (the HIP engine).  Raises if it is missing: no fallback."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64 (same SONAME), and a
        # process that also uses torch.cuda / RCCL must bind this library to that copy.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        L.k10s_last_error.restype = ctypes.c_char_p
        L.k10s_version.restype = ctypes.c_char_p
        L.k10s_engine_create.restype = ctypes.c_void_p
        L.k10s_engine_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ReplicaParams), ctypes.c_uint32,
                                         ctypes.POINTER(Capacities), ctypes.c_int32]
        L.k10s_engine_destroy.argtypes = [ctypes.c_void_p]
        L.k10s_engine_create_bulk.restype = ctypes.c_void_p
        L.k10s_engine_create_bulk.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64,
                                              ctypes.POINTER(ReplicaParams), ctypes.c_uint32,
                                              ctypes.POINTER(Capacities), ctypes.c_int32]
        L.k10s_engine_reset.argtypes = [ctypes.c_void_p]
        L.k10s_engine_reset.restype = ctypes.c_int32
        L.k10s_engine_run.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_uint64, ctypes.POINTER(ctypes.c_double)]
        L.k10s_engine_run.restype = ctypes.c_int32
        L.k10s_engine_step_async.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                             ctypes.c_uint64]
        L.k10s_engine_step_async.restype = ctypes.c_int32
        L.k10s_engine_sync.argtypes = [ctypes.c_void_p]
        L.k10s_engine_sync.restype = ctypes.c_int32
        L.k10s_schedule_one_batch.restype = ctypes.c_int32
        L.k10s_schedule_one_batch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32, ctypes.c_uint32] + \
            [ctypes.c_void_p] * 2 + [ctypes.c_double, ctypes.c_uint32] + [ctypes.c_void_p] * 3
        L.k10s_score_batch.restype = ctypes.c_int32
        L.k10s_score_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_double, ctypes.c_uint64] + \
            [ctypes.c_void_p] * 2
        L.k10s_scheduler_create.restype = ctypes.c_void_p
        L.k10s_scheduler_create.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32]
        L.k10s_scheduler_destroy.argtypes = [ctypes.c_void_p]
        L.k10s_scheduler_schedule.restype = ctypes.c_int32
        L.k10s_scheduler_schedule.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] + [ctypes.c_void_p] * 2 + \
            [ctypes.c_double, ctypes.c_uint32] + [ctypes.c_void_p] * 2
        _lib = L
    return _lib


class Engine(EngineBase):
    """A batch of independent kubernetriks replicas on one MI355X (one wavefront per replica)."""

    def __init__(self, scenario: str, n_replicas: int, params: Optional[Sequence[ReplicaParams]] = None,
                 caps: Optional[Capacities] = None, device: int = 0, pods_blob: Optional[bytes] = None):
        """pods_blob: optional binary create_pod block (scenario.scenario_bulk / k10s_engine_create_bulk)."""
        L = lib()
        self._L = L
        self._fn = _decl(L, "k10s_engine_")
        self.n_replicas = n_replicas
        parr = None
        if params is not None:
            parr = (ReplicaParams * n_replicas)(*params)
        blob = pods_blob or b""
        h = L.k10s_engine_create_bulk(scenario.encode(), blob if pods_blob else None, len(blob), parr, n_replicas,
                                      ctypes.byref(caps) if caps else None, device)
        if not h:
            raise RuntimeError("k10s_engine_create failed: " + L.k10s_last_error().decode())
        self._h = h

    def _last_error(self) -> str:
        return self._L.k10s_last_error().decode()

    def close(self):
        if getattr(self, "_h", None):
            self._L.k10s_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def reset(self):
        self._check(self._L.k10s_engine_reset(self._h))

    def run(self, mode: int = RUN_UNTIL_ALL_FINISHED, until_time: float = 0.0, max_time: float = 1e12,
            max_events_per_launch: int = 0) -> float:
        ms = ctypes.c_double()
        self._forget_names()
        self._check(self._L.k10s_engine_run(self._h, mode, until_time, max_time, max_events_per_launch,
                                            ctypes.byref(ms)))
        return ms.value

    def run_until_all_finished(self, max_time: float = 1e12, max_events_per_launch: int = 0) -> float:
        return self.run(RUN_UNTIL_ALL_FINISHED, 0.0, max_time, max_events_per_launch)

    def step_until_time(self, t: float, max_events_per_launch: int = 0) -> float:
        return self.run(RUN_UNTIL_TIME, t, 1e300, max_events_per_launch)

    def profile(self):
        """Per-replica cycle attribution (K10S_PROF variant builds; zeros otherwise): a list of
        dicts with the loop phases (loop/select/consume/dispatch/cycle/scan/scans/bounds, and in
        profiling builds aqpop/heappop/nheappop) and, in profiling builds, per event kind
        "kind_cycles" / "kind_count" lists."""
        self._L.k10s_engine_profile_width.restype = ctypes.c_uint32
        w = int(self._L.k10s_engine_profile_width())
        buf = (ctypes.c_uint64 * (self.n_replicas * w))()
        self._L.k10s_engine_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        self._L.k10s_engine_profile.restype = ctypes.c_int32
        self._check(self._L.k10s_engine_profile(self._h, buf))
        keys = ["loop", "select", "consume", "dispatch", "cycle", "scan", "scans", "bounds", "aqpop", "heappop",
                "nheappop", "emit", "nemit", "aqpush", "win_front", "win_apply"]
        out = []
        for r in range(self.n_replicas):
            row = list(buf[r * w:(r + 1) * w])
            d = dict(zip(keys, row[:min(w, 16)]))
            if w > 16:
                nk = (w - 16) // 2
                d["kind_cycles"] = row[16:16 + nk]
                d["kind_count"] = row[16 + nk:16 + 2 * nk]
            out.append(d)
        return out

    def step_async(self, mode: int, until_time: float, max_time: float, budget: int):
        self._check(self._L.k10s_engine_step_async(self._h, mode, until_time, max_time, budget))

    def sync(self):
        self._forget_names()
        self._check(self._L.k10s_engine_sync(self._h))


class Scheduler:
    """Host-buffer schedule_one surface (k10s_scheduler_*): R problems of n_nodes name-ordered
    nodes each, numpy in / numpy out.  Mirrors PodSchedulingAlgorithm::schedule_one
    (src/core/scheduler/interface.rs:14-23) with node indices instead of names."""

    def __init__(self, max_nodes: int, max_problems: int, device: int = 0):
        L = lib()
        self._L = L
        h = L.k10s_scheduler_create(max_nodes, max_problems, device)
        if not h:
            raise RuntimeError("k10s_scheduler_create failed: " + L.k10s_last_error().decode())
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.k10s_scheduler_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def schedule(self, alloc_cpu, alloc_ram, req_cpu, req_ram, present_bits=None, weight: float = 1.0):
        """alloc_cpu u32[R, N], alloc_ram u64[R, N], req_* [R], present_bits u64[R, ceil(N/64)] or None.
        Returns (node_idx i32[R] (-1 on error), status i32[R] = K10S_SCHED_*)."""
        import numpy as np
        cpu = np.ascontiguousarray(alloc_cpu, dtype=np.uint32)
        ram = np.ascontiguousarray(alloc_ram, dtype=np.uint64)
        R, N = cpu.shape
        rc = np.ascontiguousarray(req_cpu, dtype=np.uint32)
        rr = np.ascontiguousarray(req_ram, dtype=np.uint64)
        bits = None if present_bits is None else np.ascontiguousarray(present_bits, dtype=np.uint64)
        if ram.shape != (R, N) or rc.shape != (R,) or rr.shape != (R,) or \
                (bits is not None and bits.shape != (R, (N + 63) // 64)):
            raise ValueError("shape mismatch")
        out_n = np.empty(R, dtype=np.int32)
        out_s = np.empty(R, dtype=np.int32)
        rcode = self._L.k10s_scheduler_schedule(self._h, cpu.ctypes.data, ram.ctypes.data,
                                                None if bits is None else bits.ctypes.data, N, rc.ctypes.data,
                                                rr.ctypes.data, weight, R, out_n.ctypes.data, out_s.ctypes.data)
        if rcode != 0:
            raise RuntimeError(f"k10s_scheduler_schedule: {rcode}: " + self._L.k10s_last_error().decode())
        return out_n, out_s


def version() -> str:
    return lib().k10s_version().decode()
