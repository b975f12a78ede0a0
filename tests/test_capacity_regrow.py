"""Engine capacities that the reference does not have, regrown.

The reference's event queue (dslab-core's BinaryHeap), active queue and unschedulable map
(scheduler.rs:45, 49) are unbounded; the engine sizes each replica's heap and queues ahead of time
(k10s_capacities.event_heap / active_queue / unschedulable).  A replica that outgrows one stops with
K10S_ERR_HEAP_FULL / K10S_ERR_QUEUE_FULL, and k10s_engine_run / k10s_engine_sync recompile the batch
with the exhausted capacity doubled and replay every call since initialize (k10s_host.cpp regrow),
like the generated-name universes (tests/test_name_bound.py).  These tests start from ONE-entry
capacities, so the first events already overflow them, and compare against the oracle bit for bit
through run-to-completion, stepping, budgeted launches, several replicas and (GPU) the asynchronous
step + sync path; one GPU case fills more than half of the device so the regrown batch has to take
the old batch's place.
"""
import pytest

import gen
import oracle_bridge as ob
import parity
import scenarios as sc
from hostcheck_bridge import HostEngine
from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED, RUN_UNTIL_TIME

ERR_HEAP_FULL, ERR_QUEUE_FULL, ERR_NAME_BOUND = 100, 101, 102


def _gpu_engine():
    from kubernetriks_amd.native import Engine
    return Engine


BACKENDS = [
    pytest.param("host", id="host"),
    pytest.param("gpu", id="gpu", marks=pytest.mark.gpu),
]


def engine_cls(backend):
    return HostEngine if backend == "host" else _gpu_engine()


def tiny_caps(heap=1, queue=1):
    caps = parity.parity_caps(True, gauges=parity.GAUGE_ROWS)
    caps.event_heap = heap
    caps.active_queue = queue
    caps.unschedulable = queue
    return caps


def _oracle(scn, mode=RUN_UNTIL_ALL_FINISHED, until=None, max_time=20000.0):
    o = ob.OracleSim(scn, log=True, gauges=parity.GAUGE_ROWS)
    st = o.run_until_all_finished(max_time) if mode == RUN_UNTIL_ALL_FINISHED else o.step_until_time(until)
    od = o.result(placements=True, log=True)
    od["status_name"] = parity.ORACLE_STATUS[st] if not od["panicked"] else "error"
    return od


SCENARIOS = [
    ("fuzz_3", lambda: gen.random_scenario(3)),
    ("fuzz_8_removals", lambda: gen.random_scenario(8, n_pods=120)),
    ("fuzz_4_ca", lambda: gen.random_scenario(4, ca=True)),
    ("node_remove_while_running", sc.sc_node_remove_while_running),
]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("name,make", SCENARIOS, ids=[s[0] for s in SCENARIOS])
def test_one_entry_heap_and_queues_regrow_to_the_oracle(backend, name, make):
    scn = make()
    od = _oracle(scn)
    eng = engine_cls(backend)(scn, 1, caps=tiny_caps())
    eng.run_until_all_finished(20000.0)
    assert parity.compare(od, eng) == [], name
    caps, regrows = eng.capacities
    assert regrows >= 2, (name, regrows)
    assert caps["event_heap"] > 1 and caps["active_queue"] > 1 and caps["unschedulable"] > 1, caps
    assert eng.results()[0]["error_code"] not in (ERR_HEAP_FULL, ERR_QUEUE_FULL)


@pytest.mark.parametrize("backend", BACKENDS)
def test_regrow_through_stepping_and_budgets(backend):
    """The HPA scenario (tests/test_hpa.rs) with one-entry heap and queues AND a one-name pod-group
    universe: every step_until_time checkpoint (budgeted launches of 7 events, two replicas) equals
    the oracle; each regrow replays the earlier steps."""
    caps = tiny_caps()
    caps.group_name_bound = 1
    scn = sc.sc_hpa()
    o = ob.OracleSim(scn, log=True, gauges=parity.GAUGE_ROWS)
    eng = engine_cls(backend)(scn, 2, caps=caps)
    for t in (61.0, 450.0, 781.0, 1200.0):
        o.step_until_time(t)
        eng.step_until_time(t, 7)
        od = o.result(placements=True, log=True)
        od["status_name"] = parity.ORACLE_STATUS[4] if not od["panicked"] else "error"
        for r in range(2):
            assert parity.compare(od, eng, r=r) == [], (t, r)
    c, regrows = eng.capacities
    assert regrows >= 3 and c["group_name_bound"] >= 16 and c["event_heap"] > 1, (c, regrows)
    assert eng.group_sizes(0)["pod_group_1"][0] == 14


@pytest.mark.parametrize("backend", BACKENDS)
def test_regrow_keeps_unaffected_replicas_identical(backend):
    """Several replicas, seed-perturbed: the batch regrows for the replicas that overflow and every
    replica ends equal to the same batch run at default capacities."""
    from kubernetriks_amd.native import ReplicaParams  # noqa: F401
    scn = gen.random_scenario(11, n_pods=100)
    E = engine_cls(backend)
    ref = E(scn, 4, caps=parity.parity_caps(True))
    ref.run_until_all_finished(20000.0)
    eng = E(scn, 4, caps=tiny_caps(heap=8, queue=4))
    eng.run_until_all_finished(20000.0)
    assert eng.capacities[1] >= 1
    for r in range(4):
        a, b = ref.results()[r], eng.results()[r]
        assert a["counters"] == b["counters"] and parity.feq(a["time"], b["time"]), r
        assert ref.placements(r) == eng.placements(r), r


@pytest.mark.gpu
def test_async_step_and_sync_regrow_gpu():
    """k10s_engine_step_async records single-launch calls and k10s_engine_sync regrows;
    driven step by step with a one-name universe and one-entry queues, the result equals the oracle."""
    Engine = _gpu_engine()
    caps = tiny_caps()
    caps.group_name_bound = 1
    scn = sc.sc_hpa()
    od = _oracle(scn, mode=RUN_UNTIL_TIME, until=1200.0)
    od["status_name"] = parity.ORACLE_STATUS[4] if not od["panicked"] else "error"
    eng = Engine(scn, 1, caps=caps)
    # budgeted single launches (50 events each); a launch after the replica reached the time finds no
    # work and changes nothing, so a fixed count past the ~2,000 events of the scenario is exact
    for _ in range(300):
        eng.step_async(RUN_UNTIL_TIME, 1200.0, 1e300, 50)
        eng.sync()
    assert parity.compare(od, eng) == []
    c, regrows = eng.capacities
    assert regrows >= 3 and c["group_name_bound"] >= 16, (c, regrows)


@pytest.mark.gpu
def test_regrow_in_place_near_the_memory_limit_gpu():
    """a batch using more than half of the free device memory regrows in the
    old batch's place (core_create's reclaim) instead of failing; results equal the oracle."""
    import torch
    Engine = _gpu_engine()
    free_b, _ = torch.cuda.mem_get_info(0)
    scn = gen.random_scenario(3)
    od = _oracle(scn)
    # inflate each replica with a large placement log so R replicas take ~60 % of the free memory
    caps = tiny_caps()
    caps.placement_log = 1 << 24   # 16 M entries x 24 B = 384 MiB per replica
    one = Engine(scn, 1, caps=caps)
    per = one.replica_bytes
    del one
    R = max(2, int(0.6 * free_b) // per)
    eng = Engine(scn, R, caps=caps)
    eng.run_until_all_finished(20000.0)
    c, regrows = eng.capacities
    assert regrows >= 1, regrows
    for r in (0, R - 1):
        assert parity.compare(od, eng, r=r) == [], r
