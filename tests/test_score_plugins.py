"""Score plugins of the default profile (k10s_replica_params.score_plugins): LeastAllocatedResources
(the reference's, plugin.rs:52-63) and MostAllocatedResources — an opt-in extension the reference
registry (plugin.rs:13-23) does not have.  PARITY UNPINNED for MostAllocated: the only checker is the
oracle's restatement of the definition (oracle/oracle.cpp most_allocated_score); the
engine must match it bit for bit, on the host build here and on the GPU.  The default (bit 0 only)
is the reference path and is what every other parity test runs.
"""
import pytest

import gen
import oracle_bridge as ob
import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd.native import SCORE_LEAST_ALLOCATED, SCORE_MOST_ALLOCATED
from kubernetriks_amd.scenario import (GenericClusterTrace, GenericWorkloadTrace, Node, Pod, SimulationConfig,
                                       scenario_text)


def _gpu_engine():
    from kubernetriks_amd.native import Engine
    return Engine


BACKENDS = [pytest.param("host", id="host"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]


def engine_cls(backend):
    return HostEngine if backend == "host" else _gpu_engine()


def with_plugins(scn: str, plugins: int, w_la: float = None, w_ma: float = None) -> str:
    """The scenario text with the profile's score plugins set (config lines after the header)."""
    head, rest = scn.split("\n", 1)
    extra = [f"config score_plugins {plugins}"]
    if w_la is not None:
        rest = "\n".join(l for l in rest.split("\n") if not l.startswith("config score_weight "))
        extra.append(f"config score_weight {w_la!r}")
    if w_ma is not None:
        extra.append(f"config most_allocated_weight {w_ma!r}")
    return head + "\n" + "\n".join(extra) + "\n" + rest


def ma(cc, ac, cr, ar, rc, rr):
    """MostAllocatedResources in Python floats (the definition the oracle and engine restate)."""
    return (float((cc - ac + rc) % (1 << 32)) * 100.0 / float(cc) +
            float((cr - ar + rr) % (1 << 64)) * 100.0 / float(cr)) / 2.0


def test_most_allocated_packs_where_least_allocated_spreads():
    """Two equal empty nodes and small pods: LeastAllocated alternates, MostAllocated keeps filling
    the node that already holds pods (the highest (used + request) / capacity)."""
    c = GenericClusterTrace()
    for nm in ("node_a", "node_b"):
        c.create_node(0.0, Node(nm, 8000, 16 << 30))
    w = GenericWorkloadTrace()
    for i in range(6):
        w.create_pod(1.0 + 20.0 * i, Pod(f"pod_{i}", 1000, 1 << 30, 1000.0))
    base = scenario_text(SimulationConfig(), c, w)
    placed = {}
    for plugins in (1, 2):
        od, eng = parity.run_pair(HostEngine, with_plugins(base, plugins))
        assert parity.compare(od, eng) == []
        placed[plugins] = [node for _, node, _ in eng.placements(0)]
    assert len(set(placed[1])) == 2
    assert len(set(placed[2])) == 1          # every pod on one node (ties: last name first)
    # the second pod's MostAllocated score on the used node beats the empty one
    used = ma(8000, 7000, 16 << 30, 15 << 30, 1000, 1 << 30)
    empty = ma(8000, 8000, 16 << 30, 16 << 30, 1000, 1 << 30)
    assert used > empty


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed", range(8))
def test_plugin_sets_match_oracle(backend, seed):
    """Random clusters (mixed node sizes, zero requests, removals, re-created names, conditional
    moves) under MostAllocated alone and LeastAllocated + MostAllocated with odd weights."""
    plugins = (SCORE_MOST_ALLOCATED, SCORE_LEAST_ALLOCATED | SCORE_MOST_ALLOCATED)[seed % 2]
    w_la, w_ma = [(None, None), (0.37, 1.9), (1.0, -2.5), (2.0, 0.0)][seed % 4]
    scn = with_plugins(gen.random_scenario(300 + seed, n_pods=90, n_nodes=7, same_nodes=False,
                                           ca=(seed % 3 == 0)), plugins, w_la, w_ma)
    od, eng = parity.run_pair(engine_cls(backend), scn, max_time=40000.0)
    assert parity.compare(od, eng) == [], (seed, plugins)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed", range(8))
def test_plugin_sets_wide_match_oracle(backend, seed):
    """The same profiles over 70-200 mixed-size nodes (two to four 64-lane scan steps of the plugin
    kernel's scan), 300 pods, removals on even seeds."""
    plugins = (SCORE_MOST_ALLOCATED, SCORE_LEAST_ALLOCATED | SCORE_MOST_ALLOCATED)[seed % 2]
    w_la, w_ma = [(None, None), (0.37, 1.9), (1.0, -2.5), (2.0, 0.0)][seed % 4]
    n_nodes = 70 + (seed * 37) % 131
    scn = with_plugins(gen.random_scenario(500 + seed, n_pods=300, n_nodes=n_nodes, horizon=1200.0,
                                           same_nodes=False, removals=(seed % 2 == 0), ca=(seed % 3 == 0)),
                       plugins, w_la, w_ma)
    od, eng = parity.run_pair(engine_cls(backend), scn, max_time=40000.0)
    assert parity.compare(od, eng) == [], (seed, plugins)


@pytest.mark.parametrize("backend", BACKENDS)
def test_per_replica_plugin_sweep(backend):
    """One batch, replicas differing only in score plugins / weights (k10s_replica_params), each
    equal to the oracle on the scenario with that profile."""
    scn = gen.random_scenario(77, n_pods=120, n_nodes=9, same_nodes=False)
    E = engine_cls(backend)
    probe = E(scn, 1)
    base = probe.default_params()
    combos = [(1, 1.0, 1.0), (2, 1.0, 1.0), (3, 1.0, 1.0), (3, 0.5, 2.0), (2, 1.0, -1.0), (1, 3.0, 1.0)]
    params = []
    for r, (pl, wl_, wm) in enumerate(combos):
        p = type(base).from_buffer_copy(base)
        p.score_plugins, p.score_weight, p.most_allocated_weight = pl, wl_, wm
        p.seed = base.seed + r
        params.append(p)
    eng = E(scn, len(params), params=params, caps=parity.parity_caps(False))
    eng.run_until_all_finished(40000.0)
    for r, (pl, wl_, wm) in enumerate(combos):
        o = ob.OracleSim(with_plugins(scn, pl, wl_, wm))
        st = o.run_until_all_finished(40000.0)
        od = o.result(placements=True)
        od["status_name"] = parity.ORACLE_STATUS[st]
        assert parity.compare(od, eng, r=r, log=False) == [], r


def test_invalid_plugin_sets_are_refused():
    scn = gen.random_scenario(1)
    for bad in (0, 4, 7):
        with pytest.raises(ValueError):
            HostEngine(with_plugins(scn, bad))
    probe = HostEngine(scn, 1)
    p = type(probe.default_params()).from_buffer_copy(probe.default_params())
    p.score_plugins = 0
    with pytest.raises(ValueError):
        HostEngine(scn, 1, params=[p])
    with pytest.raises(Exception):
        ob.OracleSim(with_plugins(scn, 0))


def test_config_profile_extension_key():
    d = {"scheduling_cycle_interval": 10.0, "as_to_ps_network_delay": 0.05, "ps_to_sched_network_delay": 0.01,
         "sched_to_as_network_delay": 0.02, "as_to_node_network_delay": 0.15, "as_to_ca_network_delay": 0.3,
         "as_to_hpa_network_delay": 0.4}
    assert SimulationConfig.from_dict(d).score_plugins == 1
    d["scheduler_score_plugins"] = [{"name": "MostAllocatedResources", "weight": 2.0},
                                    {"name": "LeastAllocatedResources", "weight": 0.5}]
    c = SimulationConfig.from_dict(d)
    assert (c.score_plugins, c.score_weight, c.most_allocated_weight) == (3, 0.5, 2.0)
    text = scenario_text(c, GenericClusterTrace(), GenericWorkloadTrace())
    assert "config score_plugins 3" in text and "config most_allocated_weight 2.0" in text
    for bad in ([{"name": "BalancedAllocation", "weight": 1.0}],
                [{"name": "LeastAllocatedResources", "weight": 1.0}] * 2, []):
        d["scheduler_score_plugins"] = bad
        with pytest.raises(ValueError):
            SimulationConfig.from_dict(d)
