"""The scheduling cycle's tiles (k10s_engine.h fit_tile / run_scheduling_cycle_t): after a cycle with a
failed attempt, the cycle pops K10S_TILE (8) pods at a time, tests in one shared read of the packed
node cache whether each fits some node, fails the ones that fit nowhere without a scan (exact: nothing
is pushed onto the action queue during a cycle, scheduler.rs:261-330, and a reservation only lowers a
node's allocatable, 118-123), and schedules the others one at a time by the exact scan.

Adversarial cases against the oracle, bit for bit (counters, clock, estimators, every placement and
the whole event log), on the host build and the GPU:
* every pod wants the same node (identical nodes, identical pods, ties to the last index);
* pods that fit nowhere mixed with pods that fit, and tiles in which only later pods fit after
  earlier ones took the room;
* cycles of fewer than, exactly and more than 8 pods (a tile never spans two cycles);
* node removal and re-creation between cycles;
* a removed pod inside a tile (skipped like the loop's `continue`);
* weight != 1, and zero requests, which stay on the serial path;
* the conditional move (pods stay unschedulable) and move-all.
A backlog case also checks that the tiles replaced scans (nodes_read below attempts x nodes)."""
import random

import pytest

import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd.scenario import (GenericClusterTrace, GenericWorkloadTrace, Node, Pod, SimulationConfig,
                                       scenario_text)

BACKENDS = [pytest.param("host", id="host"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]
GIB = 1 << 30


def _engine(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


def backlog_scenario(seed: int, n_nodes: int = 24, n_pods: int = 300, identical: bool = False, cond_move: bool = False,
                     cycle: float = 10.0, removals: bool = False, weight: float = 1.0, zero_every: int = 0,
                     huge_every: int = 0, pod_removals: bool = False, bursts: bool = True) -> str:
    rng = random.Random(seed)
    cfg = SimulationConfig()
    cfg.enable_unscheduled_pods_conditional_move = cond_move
    cfg.scheduling_cycle_interval = cycle
    cfg.score_weight = weight
    c = GenericClusterTrace()
    for k in range(n_nodes):
        cpu = 8000 if identical else rng.choice([4000, 8000, 16000])
        ram = 32 * GIB if identical else rng.choice([16, 32, 64]) * GIB
        c.create_node(0.0, Node(f"node_{k:03d}", cpu, ram))
    if removals:   # half the nodes leave mid-run, a quarter come back under the same names
        for k in range(0, n_nodes, 2):
            c.remove_node(200.0 + 3 * k, f"node_{k:03d}")
        for k in range(0, n_nodes, 4):
            c.create_node(400.0 + 5 * k, Node(f"node_{k:03d}", 8000, 32 * GIB))
    w = GenericWorkloadTrace()
    for i in range(n_pods):
        t = float(rng.randint(0, 8) * 25 if bursts else rng.randint(0, 600))
        if identical:
            cpu, ram = 3000, 12 * GIB
        else:
            cpu = rng.choice([500, 1000, 2000, 3000, 6000])
            ram = int(rng.uniform(0.2, 0.7) * 32 * GIB)
        if zero_every and i % zero_every == 0:
            cpu, ram = 0, 0
        if huge_every and i % huge_every == 1:
            cpu, ram = 20000, 100 * GIB   # fits no node
        w.create_pod(t, Pod(f"pod_{i:04d}", cpu, ram, float(rng.randint(20, 400))))
        if pod_removals and i % 17 == 3:
            w.remove_pod(t + rng.choice([0.0, 5.0, 30.0, 120.0]), f"pod_{i:04d}")
    return scenario_text(cfg, c, w)


CASES = {
    "backlog": dict(seed=1),
    "identical": dict(seed=2, identical=True),
    "identical_cond_move": dict(seed=3, identical=True, cond_move=True),
    "fit_nowhere": dict(seed=4, huge_every=5),
    "removals": dict(seed=5, removals=True),
    "pod_removals": dict(seed=6, pod_removals=True),
    "short_cycles": dict(seed=7, cycle=1.0, bursts=False),
    "long_cycles": dict(seed=8, cycle=30.0, n_pods=500),
    "weight": dict(seed=9, weight=0.37),
    "zero_requests": dict(seed=10, zero_every=7),
    "cond_move": dict(seed=11, cond_move=True),
    "few_nodes": dict(seed=12, n_nodes=3, n_pods=120),
}


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("case", sorted(CASES))
def test_cycle_tiles_match_oracle(backend, case):
    scn = backlog_scenario(**CASES[case])
    od, eng = parity.run_pair(_engine(backend), scn, max_time=1e6)
    assert parity.compare(od, eng) == [], case
    k = eng.results()[0]["counters"]
    assert k["attempts"] > k["placements"] > 0, case   # failed attempts: the tiles run


@pytest.mark.parametrize("backend", BACKENDS)
def test_tiles_replace_failed_scans(backend):
    """In the backlog regime the failed attempts cost one shared read per tile, not a scan each."""
    scn = backlog_scenario(21, n_nodes=64, n_pods=800)
    od, eng = parity.run_pair(_engine(backend), scn, max_time=1e6, log=False)
    assert parity.compare(od, eng, log=False) == []
    k = eng.results()[0]["counters"]
    fails = k["attempts"] - k["placements"]
    assert fails > 2 * k["placements"]
    # every placement still scans the whole cache; the failed attempts read far less than one each
    read_by_fails = k["nodes_read"] - 64 * k["placements"]
    assert read_by_fails < 0.5 * 64 * fails, (read_by_fails, fails)
