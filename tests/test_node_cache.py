"""The scheduler's node cache in its two layouts (k10s_engine.h nc_*, k10s_capacities.node_cache):
packed (one u64 per node, cpu << 40 | ram: 8 B per node and scan) wherever every node definition
fits (cpu < 2^24, ram < 2^40) and no replica needs the wide SoA, else wide (u32 cpu + u64 ram).
Both layouts run the same scenarios bit-exactly against the oracle; the wide one on the GPU is the
second kernel copy (k10s_kernels_plugins.hip) with LeastAllocated-only replicas.  The packed
field edges (cpu 2^24 - 1, ram 2^40 - 1) are exercised with nodes exactly at the limits."""
import pytest

import gen
import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd import workloads as wl
from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED, RUN_UNTIL_TIME
from kubernetriks_amd.scenario import GenericClusterTrace, GenericWorkloadTrace, Node, Pod, SimulationConfig, scenario_text

BACKENDS = [pytest.param("host", id="host"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]
WIDE = 1


def engine_cls(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


SEEDS = list(range(0, 24))


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed", SEEDS)
def test_wide_layout_matches_oracle(backend, seed):
    """The fuzz scenarios (packed by default in every other test) forced onto the wide layout."""
    kw = dict(ca=(seed % 3 == 1), hpa=(seed % 4 == 2))
    mode = RUN_UNTIL_TIME if kw["hpa"] else RUN_UNTIL_ALL_FINISHED
    od, eng = parity.run_pair(engine_cls(backend), gen.random_scenario(seed, **kw), mode=mode, until=3000.0,
                              max_time=20000.0, node_cache=WIDE)
    assert eng.node_entry_bytes == 12
    assert parity.compare(od, eng) == [], seed


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed", range(10_000, 10_012))
def test_wide_layout_multi_step_scans_match_oracle(backend, seed):
    """test_engine_parity's wide random scenarios (50-200 nodes: one to four 64-lane scan steps)
    forced onto the wide layout."""
    import random
    rng = random.Random(seed)
    kw = dict(ca=(seed % 3 == 1), hpa=(seed % 4 == 2), removals=(seed % 2 == 0))
    scn = gen.random_scenario(seed, n_pods=rng.choice([200, 400, 800]), n_nodes=rng.randint(50, 200),
                              horizon=1200.0, **kw)
    mode = RUN_UNTIL_TIME if kw["hpa"] else RUN_UNTIL_ALL_FINISHED
    od, eng = parity.run_pair(engine_cls(backend), scn, mode=mode, until=3000.0, max_time=20000.0,
                              node_cache=WIDE)
    assert eng.node_entry_bytes == 12
    assert parity.compare(od, eng) == [], seed


def edge_scenario(cpu: int, ram: int, seed: int = 0) -> str:
    """Nodes at (and one step below) the given capacities, pods sized so nodes fill up, release and
    refill: allocatable crosses every field value from 0 to the capacity."""
    import random
    rng = random.Random(seed)
    c = GenericClusterTrace()
    for k in range(6):
        c.create_node(0.0, Node(f"node_{k}", cpu - (k % 2), ram - (k % 3)))
    w = GenericWorkloadTrace()
    for i in range(120):
        rc = rng.choice([1, cpu // 7, cpu // 3, cpu // 2 + 1, cpu - 1])
        rr = rng.choice([1, ram // 5, ram // 3, ram // 2 + 1, ram - 2])
        w.create_pod(float(rng.randint(0, 300)), Pod(f"pod_{i:03d}", max(rc, 1), max(rr, 1), float(rng.randint(5, 200))))
    return scenario_text(SimulationConfig(), c, w)


@pytest.mark.parametrize("backend", BACKENDS)
def test_packed_field_limits(backend):
    """cpu 2^24 - 1 and ram 2^40 - 1 are packable and run bit-exactly; one more unit of either makes
    the engine fall back to the wide layout, also bit-exact."""
    E = engine_cls(backend)
    for cpu, ram, nb in (((1 << 24) - 1, (1 << 40) - 1, 8), (1 << 24, (1 << 40) - 1, 12), ((1 << 24) - 1, 1 << 40, 12)):
        od, eng = parity.run_pair(E, edge_scenario(cpu, ram), max_time=1e6)
        assert eng.node_entry_bytes == nb, (cpu, ram)
        assert parity.compare(od, eng) == [], (cpu, ram)
        assert eng.results()[0]["counters"]["placements"] > 50


@pytest.mark.parametrize("backend", BACKENDS)
def test_layout_choice(backend):
    """Packed for the bench's Alibaba-like clusters; wide for the pruned scan, for a replica with a
    score plugin beyond LeastAllocated, and on request."""
    E = engine_cls(backend)
    c, w = wl.c3_traces(n_nodes=64, n_pods=100, arrival_window=50.0, seed=3)
    scn = scenario_text(SimulationConfig(), c, w)
    assert E(scn, 2).node_entry_bytes == 8
    assert E(scn, 2, caps=parity.parity_caps(False, pruned=1)).node_entry_bytes == 12
    caps = parity.parity_caps(False)
    caps.node_cache = WIDE
    assert E(scn, 2, caps=caps).node_entry_bytes == 12
    params = wl.replica_params(E(scn, 1).default_params(), 2)
    params[1].score_plugins = 3
    params[1].most_allocated_weight = 1.0
    assert E(scn, 2, params=params).node_entry_bytes == 12
    assert E(scn, 2).replica_bytes < E(scn, 2, caps=caps).replica_bytes   # 8 B/node and no capacity SoA


def signed_time_scenario(t0: float) -> str:
    """Pods created at t0 (and a little after), so the trace holds timestamps of t0's sign."""
    c = GenericClusterTrace()
    for k in range(4):
        c.create_node(0.0, Node(f"node_{k}", 8000, 16 << 30))
    w = GenericWorkloadTrace()
    for i in range(40):
        w.create_pod(t0 + (i % 5) * 0.5 if t0 else t0, Pod(f"pod_{i:03d}", 500 + 100 * (i % 7), (1 + i % 5) << 28,
                                                           float(10 + 7 * (i % 9))))
    return scenario_text(SimulationConfig(), c, w)


def _set_config(text: str, key: str, value: float) -> str:
    """Rewrite one `config <key> <value>` line (or a key of the hpa_config / ca_config line)."""
    out = []
    for line in text.splitlines():
        f = line.split()
        if f[:2] == ["config", key]:
            line = f"config {key} {value!r}"
        elif f and f[0] in ("hpa_config", "ca_config") and key in f:
            f[f.index(key) + 1] = repr(value)
            line = " ".join(f)
        out.append(line)
    return "\n".join(out) + "\n"


@pytest.mark.parametrize("backend", BACKENDS)
def test_signed_event_times_take_the_general_key(backend):
    """The default kernel keys event times by their bit pattern (k10s_common.h total_key), exact only
    for times that are >= 0: -0.0 trace timestamps keep the packed layout (default copy) and match the
    oracle; a replica with a negative network delay runs the second copy (wide layout), which checks
    every emission's delay like dslab-core."""
    E = engine_cls(backend)
    od, eng = parity.run_pair(E, signed_time_scenario(-0.0), max_time=1e6)
    assert eng.node_entry_bytes == 8
    assert parity.compare(od, eng) == []
    scn = signed_time_scenario(3.0)
    params = wl.replica_params(E(scn, 1).default_params(), 2)
    assert E(scn, 2, params=params).node_entry_bytes == 8
    params[1].as_to_ps_network_delay = -0.001
    assert E(scn, 2, params=params).node_entry_bytes == 12
    params[1].as_to_ps_network_delay = float("nan")
    assert E(scn, 2, params=params).node_entry_bytes == 12


def test_negative_trace_timestamps_are_refused():
    """initialize emits every trace event at delay = its timestamp (simulator.rs:234-253) and dslab-core
    refuses a negative delay with a panic: the oracle fails in initialize, the engine refuses the
    scenario (both builds share the builder)."""
    import oracle_bridge as ob
    for t0 in (-7.25, -1e-300):
        scn = signed_time_scenario(t0)
        with pytest.raises(ValueError, match="negative"):
            ob.OracleSim(scn)
        with pytest.raises(ValueError, match="negative"):
            HostEngine(scn, 1)


def negative_delay_cases():
    """(name, scenario, mode) where some emission gets a negative delay, or a negative duration lands
    a pod's finish in storage before its start."""
    base = signed_time_scenario(3.0)
    hpa = gen.random_scenario(2, hpa=True)
    ca = gen.random_scenario(1, ca=True)
    yield "as_to_ps_delay", _set_config(base, "as_to_ps_network_delay", -0.001), RUN_UNTIL_ALL_FINISHED
    # a heap-sourced handler (the HPA / CA tick) re-emits itself into the heap with a negative delay
    yield "hpa_interval", _set_config(hpa, "scan_interval", -30.0), RUN_UNTIL_TIME
    # (the CA's re-tick uses delay 0 whenever more than the interval has passed since its last cycle,
    # cluster_autoscaler.rs:320-331: a negative interval never reaches an emission, no panic)
    yield "ca_interval", _set_config(ca, "scan_interval", -5.0), RUN_UNTIL_TIME
    # (a negative scheduling-cycle interval never reaches an emission either: the next cycle is due at
    # max(cycle duration, interval) = the cycle duration >= 0, scheduler.rs:331-333 — and with an empty
    # queue that is 0, an endless cycle at one instant in the reference too; not a test case)
    # negative durations: the finish self-event's delay (duration + as_to_node delay 0.152) is < 0 ...
    c = GenericClusterTrace()
    for k in range(3):
        c.create_node(0.0, Node(f"node_{k}", 8000, 16 << 30))
    w = GenericWorkloadTrace()
    for i in range(12):
        w.create_pod(1.0 + i, Pod(f"pod_{i:02d}", 1000, 1 << 30, -5.0 if i == 7 else 20.0))
    yield "duration_below_delay", scenario_text(SimulationConfig(), c, w), RUN_UNTIL_ALL_FINISHED
    # ... or >= 0, so the finish reaches storage before the start (persistent_storage.rs:313 panics)
    w = GenericWorkloadTrace()
    for i in range(12):
        w.create_pod(1.0 + i, Pod(f"pod_{i:02d}", 1000, 1 << 30, -0.1 if i == 4 else 20.0))
    yield "finish_before_start", scenario_text(SimulationConfig(), c, w), RUN_UNTIL_ALL_FINISHED


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", [c[0] for c in negative_delay_cases()])
def test_negative_delays_panic_like_dslab(backend, case):
    """dslab-core refuses an event in the past with a panic (add_event: `delay >= 0.` or panic): every
    such scenario runs the signed-time kernel copy, which checks each emission, and stops where the
    oracle panics, with the same clock, counters and event log up to that point
    (K10S_PANIC_NEGATIVE_DELAY); a finish that overtakes its start ends like the oracle too."""
    from kubernetriks_amd.native import K10S_PANIC_MISSING_POD, K10S_PANIC_NEGATIVE_DELAY
    name, scn, mode = next(c for c in negative_delay_cases() if c[0] == case)
    od, eng = parity.run_pair(engine_cls(backend), scn, mode=mode, until=2000.0, max_time=1e6)
    assert od["panicked"] == (name != "ca_interval"), od["status_name"]
    assert eng.node_entry_bytes == 12
    assert parity.compare(od, eng) == [], name
    code = eng.results()[0]["error_code"]
    if name == "ca_interval":
        assert code == 0
    elif name == "finish_before_start":
        assert "PodStartedRunning" in od["panic"] and code == K10S_PANIC_MISSING_POD
    else:
        assert "negative" in od["panic"] and code == K10S_PANIC_NEGATIVE_DELAY
