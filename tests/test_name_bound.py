"""Generated names without a bound, as in the reference.

The reference names the HPA's pods "{group}_{total_created}" (kube_horizontal_pod_autoscaler.rs:178-182,
api_server.rs:421) and the cluster autoscaler's nodes "{group}_{k}" with no limit.  The engine ranks
every name of a run ahead of time (name rank = index), so it compiles a finite universe per group; a
replica that would outgrow it stops with K10S_ERR_NAME_BOUND, and the engine then recompiles the
batch with that universe doubled and replays every run call since initialize (include/k10s.h
k10s_engine_name_bounds).  These tests run at the DEFAULT capacities (no parity override) on the five
random scenarios whose HPA churn outgrew the default universe in round 4's 2,000-seed sweep, and on
forced one-name universes through multi-call histories (stepping, budgeted launches, several
replicas), always against the oracle bit for bit.
"""
import pytest

import gen
import oracle_bridge as ob
import parity
import scenarios as sc
from hostcheck_bridge import HostEngine
from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED, RUN_UNTIL_TIME


def _gpu_engine():
    from kubernetriks_amd.native import Engine
    return Engine


BACKENDS = [
    pytest.param("host", id="host"),
    pytest.param("gpu", id="gpu", marks=pytest.mark.gpu),
]


def engine_cls(backend):
    return HostEngine if backend == "host" else _gpu_engine()


# round 4's 2,000-seed fuzz sweep: these outgrew the default universe (8 x max + 64 per group)
CHURN_SEEDS = [546, 878, 898, 1106, 1530]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed", CHURN_SEEDS)
def test_hpa_churn_at_default_capacities_matches_oracle(backend, seed):
    kw = dict(ca=(seed % 3 == 1), hpa=(seed % 4 == 2))
    scn = gen.random_scenario(seed, **kw)
    E = engine_cls(backend)
    default_bound = E(scn, 1).name_bounds[0]
    od, eng = parity.run_pair(E, scn, mode=RUN_UNTIL_TIME if kw["hpa"] else RUN_UNTIL_ALL_FINISHED,
                              until=3000.0, max_time=20000.0)
    assert parity.compare(od, eng) == [], seed
    assert eng.results()[0]["error_code"] != 102
    assert eng.name_bounds[0] > default_bound, "the run was expected to outgrow the default universe"


def _stepped_pair(E, scn, caps, times, budget=0, replicas=1):
    o = ob.OracleSim(scn, log=True, gauges=parity.GAUGE_ROWS)
    eng = E(scn, replicas, caps=caps)
    for t in times:
        o.step_until_time(t)
        eng.step_until_time(t, budget)
        od = o.result(placements=True, log=True)
        od["status_name"] = parity.ORACLE_STATUS[4] if not od["panicked"] else "error"
        for r in range(replicas):
            assert parity.compare(od, eng, r=r) == [], (t, r)
    return eng


@pytest.mark.parametrize("backend", BACKENDS)
def test_one_name_group_universe_regrows_through_stepping(backend):
    """The HPA scenario (tests/test_hpa.rs) with a universe of ONE name per pod group: its five
    initial pods already exceed it, and the HPA later scales to 14; each step_until_time must equal
    the oracle, the regrown batch replaying the earlier steps (budgeted launches of 7 events)."""
    caps = parity.parity_caps(True, gauges=parity.GAUGE_ROWS)
    caps.group_name_bound = 1
    eng = _stepped_pair(engine_cls(backend), sc.sc_hpa(), caps, (61.0, 450.0, 781.0, 1200.0), budget=7, replicas=2)
    assert eng.name_bounds[0] >= 16
    assert eng.group_sizes(0)["pod_group_1"][0] == 14


@pytest.mark.parametrize("backend", BACKENDS)
def test_one_name_ca_universe_regrows(backend):
    """A cluster-autoscaler scenario with ONE name per CA node group: the second scale-up needs a
    second name; the regrown batch equals the oracle."""
    for seed in (1, 4, 7, 10):
        scn = gen.random_scenario(seed, ca=True)
        o = ob.OracleSim(scn, log=True, gauges=parity.GAUGE_ROWS)
        st = o.run_until_all_finished(20000.0)
        od = o.result(placements=True, log=True)
        od["status_name"] = parity.ORACLE_STATUS[st] if not od["panicked"] else "error"
        if od["counters"]["total_scaled_up_nodes"] < 2:
            continue
        caps = parity.parity_caps(True, gauges=parity.GAUGE_ROWS)
        caps.ca_name_bound = 1
        eng = engine_cls(backend)(scn, 1, caps=caps)
        eng.run_until_all_finished(20000.0)
        assert parity.compare(od, eng) == [], seed
        assert eng.name_bounds[1] > 1
        return
    pytest.fail("no seed scaled up twice")
