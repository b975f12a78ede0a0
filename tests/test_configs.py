"""BASELINE.json configs C2, C4 and C5 as batched parity cases: R replicas in one engine batch, each
replica compared bit-exactly (counters, estimators, clock, placements, per-pod times) with the CPU
oracle run on that replica's own scenario (its parameters + its seed-perturbed trace, materialized
on the host by workloads.replica_scenario).  Shapes are scaled down so the oracle finishes in
seconds; the full-size configs run in bench.py.

  C2  31-node default cluster (config.yaml:45-68), test_determinism-style pods, seed-perturbed
  C4  test_hpa.rs pod group + config.yaml:14-33 CA node groups, burst workload (scale-up, drain)
  C5  C3-shaped cluster with the scheduler/autoscaler parameter sweep (cycle interval, conditional
      move, network delays, CA threshold, HPA tolerance), and the same sweep over the C4 scenario
"""
import pytest

import oracle_bridge as ob
import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd import workloads as wl
from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED, RUN_UNTIL_TIME
from kubernetriks_amd.scenario import scenario_text

BACKENDS = [pytest.param("host", id="host"), pytest.param("gpu", id="gpu", marks=pytest.mark.gpu)]


def engine_cls(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


def _batch_parity(backend, parts, params_fn, R, check, mode=RUN_UNTIL_ALL_FINISHED, until=0.0, max_time=1e6,
                  parallel=False):
    cfg, c, w = parts
    E = engine_cls(backend)
    probe = E(scenario_text(cfg, c, w), 1)
    params = params_fn(probe.default_params(), R)
    eng = E(scenario_text(cfg, c, w), R, params=params, caps=parity.parity_caps(False))
    if mode == RUN_UNTIL_ALL_FINISHED:
        eng.run_until_all_finished(max_time)
    else:
        eng.step_until_time(until)
    if parallel and mode == RUN_UNTIL_ALL_FINISHED:
        import oracle_jobs
        ods = oracle_jobs.replay_many([wl.replica_scenario(cfg, c, w, params[r]) for r in check], max_time)
        for r, od in zip(check, ods):
            assert parity.compare(od, eng, r=r, log=False) == [], r
        return eng
    for r in check:
        o = ob.OracleSim(wl.replica_scenario(cfg, c, w, params[r]))
        st = o.run_until_all_finished(max_time) if mode == RUN_UNTIL_ALL_FINISHED else o.step_until_time(until)
        od = o.result(placements=True)
        od["status_name"] = parity.ORACLE_STATUS[st] if not od["panicked"] else "error"
        assert parity.compare(od, eng, r=r, log=False) == [], r
    return eng


@pytest.mark.parametrize("backend", BACKENDS)
def test_c2_default_cluster_seed_perturbed(backend):
    R = 32 if backend == "gpu" else 4
    eng = _batch_parity(backend, wl.c2_parts(n_pods=300, seed=123),
                        lambda d, n: wl.replica_params(d, n, base_seed=123, perturb=True), R,
                        check=sorted({0, 1, R // 2, R - 1}))
    res = eng.results()
    assert all(r["status"] == "finished" for r in res)
    assert len({r["counters"]["events"] for r in res}) > 1  # perturbation makes replicas differ


@pytest.mark.parametrize("backend", BACKENDS)
def test_c4_hpa_and_cluster_autoscaler_batched(backend):
    R = 24 if backend == "gpu" else 3
    eng = _batch_parity(backend, wl.c4_parts(n_batch_pods=80, seed=7),
                        lambda d, n: wl.replica_params(d, n, base_seed=7, perturb=True), R,
                        check=sorted({0, R // 2, R - 1}), mode=RUN_UNTIL_TIME, until=1500.0)
    c = eng.results()[0]["counters"]
    assert c["total_scaled_up_nodes"] > 0 and c["total_scaled_up_pods"] > 0


@pytest.mark.parametrize("backend", BACKENDS)
def test_c5_parameter_sweep_c3_shape(backend):
    R = 48 if backend == "gpu" else 8
    # replicas 0..7 cover every cycle interval with and without conditional move
    parts = (wl.SimulationConfig(),) + wl.c3_traces(n_nodes=192, n_pods=400, arrival_window=200.0, seed=11)
    _batch_parity(backend, parts, lambda d, n: wl.c5_params(d, n, base_seed=123), R,
                  check=list(range(8)) if backend == "host" else [0, 3, 5, 8, 13, 24, 31, 47])


@pytest.mark.parametrize("backend", BACKENDS)
def test_c5_parameter_sweep_over_autoscalers(backend):
    """The sweep axes that only matter with autoscalers on: CA scale-down threshold (replica // 24)
    and HPA tolerance (replica // 72), over the C4 scenario."""
    idx = [0, 24, 48, 72, 144] if backend == "host" else list(range(0, 216, 9))
    R = max(idx) + 1
    cfg, c, w = wl.c4_parts(n_batch_pods=40, seed=3)
    E = engine_cls(backend)
    probe = E(scenario_text(cfg, c, w), 1)
    allp = wl.c5_params(probe.default_params(), R, base_seed=500)
    params = [allp[i] for i in idx]
    eng = E(scenario_text(cfg, c, w), len(idx), params=params, caps=parity.parity_caps(False))
    eng.step_until_time(1500.0)
    for k in range(len(idx)):
        o = ob.OracleSim(wl.replica_scenario(cfg, c, w, params[k]))
        o.step_until_time(1500.0)
        od = o.result(placements=True)
        od["status_name"] = parity.ORACLE_STATUS[4] if not od["panicked"] else "error"
        assert parity.compare(od, eng, r=k, log=False) == [], idx[k]


# ---- the BASELINE sizes on the GPU ------------------------------------------------------------
# Full replica counts per GPU (C2: 1,024; C4: 1,024; C5: 8,192 = 65,536 / 8 GPUs) in one batch,
# with whole-batch properties (every replica terminates, the finish-hook identity
# simulation_callbacks.rs:73-76 holds, the perturbation/sweep makes replicas differ) and bit-exact
# oracle replays of replicas spread over the batch (first, last, both halves' edges).
def _identity(res):
    for r in res:
        k = r["counters"]
        assert k["terminated_pods"] == k["pods_succeeded"] + k["pods_unschedulable"] + k["pods_failed"] + \
            k["pods_removed"], r


@pytest.mark.gpu
def test_c2_at_baseline_size_gpu():
    R = 1024
    eng = _batch_parity("gpu", wl.c2_parts(n_pods=300, seed=123),
                        lambda d, n: wl.replica_params(d, n, base_seed=123, perturb=True), R,
                        check=[0, 1, 511, 512, 1022, 1023])
    res = eng.results()
    assert all(r["status"] == "finished" for r in res)
    _identity(res)
    # perturbed durations: the pod-duration estimators differ (finish times are multiples of 1000 s)
    assert len({tuple(r["estimators"]["pod_duration"][1:5]) for r in res}) > R // 4


@pytest.mark.gpu
def test_c4_at_baseline_size_gpu():
    R = 1024
    eng = _batch_parity("gpu", wl.c4_parts(n_batch_pods=80, seed=7),
                        lambda d, n: wl.replica_params(d, n, base_seed=7, perturb=True), R,
                        check=[0, 511, 1023], mode=RUN_UNTIL_TIME, until=1500.0)
    res = eng.results()
    assert sum(r["counters"]["total_scaled_up_nodes"] > 0 for r in res) == R


@pytest.mark.gpu
def test_c5_sweep_at_baseline_size_gpu():
    """One GPU's share of the 65,536-replica sweep (8,192 replicas) on 4,096-node clusters."""
    R = 8192
    parts = (wl.SimulationConfig(),) + wl.c3_traces(n_nodes=4096, n_pods=600, arrival_window=200.0, seed=11)
    # one replica of every (cycle interval x conditional move x delays x CA threshold) cell: replicas
    # 0..71 (workloads.c5_params), replayed in parallel, plus the batch's far end
    eng = _batch_parity("gpu", parts, lambda d, n: wl.c5_params(d, n, base_seed=123), R,
                        check=list(range(72)) + [4095, 8191], parallel=True)
    res = eng.results()
    assert all(r["status"] == "finished" for r in res)
    _identity(res)
    assert len({tuple(r["estimators"]["pod_queue_time"][1:5]) for r in res}) >= 8   # cycle interval x cond. move


# ---- per-replica trace lengths (k10s_replica_params.workload_prefix) ---------------------------
@pytest.mark.parametrize("backend", BACKENDS)
def test_workload_prefix_replicas_match_their_own_traces(backend):
    """Replicas that keep only the first k workload events (k spread over 0..all, including a prefix
    that cuts before the pod group and the removals) run exactly like the oracle on the shortened
    trace: ids, total_pods_in_trace and the termination rule follow the replica's own trace."""
    cfg, c, w = wl.c4_parts(n_batch_pods=60, seed=5)
    w.remove_pod(900.0, "batch_3")
    w.remove_pod(950.0, "batch_7")
    scn = scenario_text(cfg, c, w)
    E = engine_cls(backend)
    W = len(w.events)
    prefixes = [0, 1, 2, 17, W - 3, W - 1, W]
    params = wl.replica_params(E(scn, 1).default_params(), len(prefixes), base_seed=41, perturb=True)
    for p, k in zip(params, prefixes):
        p.workload_prefix = k
    eng = E(scn, len(prefixes), params=params, caps=parity.parity_caps(False))
    eng.step_until_time(2500.0)
    for r, k in enumerate(prefixes):
        o = ob.OracleSim(wl.replica_scenario(cfg, c, w, params[r]))
        o.step_until_time(2500.0)
        od = o.result(placements=True)
        od["status_name"] = parity.ORACLE_STATUS[4] if not od["panicked"] else "error"
        assert parity.compare(od, eng, r=r, log=False) == [], (r, k)
    tot = [res["counters"]["total_pods_in_trace"] for res in eng.results()]
    assert tot[0] == tot[-1] == sum(1 for e in w.events if e.kind == "create_pod")
    assert tot[1] == 0 and tot[1:] == sorted(tot[1:])   # prefix 1 keeps only the pod group
    bad = wl.replica_params(E(scn, 1).default_params(), 1)
    bad[0].workload_prefix = W + 1
    with pytest.raises(Exception):
        E(scn, 1, params=bad)


def test_c2_survey_size_host():
    """C2 at SURVEY size, CPU-sized: per-replica ceil(U * n) prefixes of one master trace."""
    parts = wl.c2_survey_parts(n_max=400, horizon=4000.0)
    eng = _batch_parity("host", parts, lambda d, n: wl.c2_survey_params(d, n, n_max=400), 4, check=[0, 1, 2, 3])
    res = eng.results()
    assert [r["counters"]["total_pods_in_trace"] for r in res] == [wl.c2_survey_prefix(r, 400) for r in range(4)]


@pytest.mark.gpu
def test_c2_at_survey_size_gpu():
    """C2 as SURVEY.md §8(d) sizes it: 1,024 replicas of the 31-node default cluster, replica r
    running the first ceil(U_r * 10,000) pods of a test_determinism-style master trace (arrivals over
    1e5 s), seed-perturbed, in one engine batch; oracle replays of the shortest, the longest and
    replicas spread over the batch."""
    R = 1024
    pre = [wl.c2_survey_prefix(r) for r in range(R)]
    check = sorted({0, 1, 511, 1023, pre.index(min(pre)), pre.index(max(pre))})
    eng = _batch_parity("gpu", wl.c2_survey_parts(), lambda d, n: wl.c2_survey_params(d, n), R, check=check)
    res = eng.results()
    assert all(r["status"] == "finished" for r in res)
    _identity(res)
    assert [r["counters"]["total_pods_in_trace"] for r in res] == pre
