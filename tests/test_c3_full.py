"""The C3 shape at its full node count (4,096 Alibaba-like nodes, BASELINE.json configs[2]) against the
oracle, replica by replica and bit for bit, in two load regimes:

* light  (wl.c3_traces): every attempt places its pod — the bench's default workload;
* backlog (wl.c3_backlog_traces, SURVEY.md §8(d) rho ~ 1): attempts fail, pods wait in the
  unschedulable map, are moved back to the action queue on every pod finish
  (scheduler.rs:235-244, 422-440) and flushed after 300 s (188-203).

The engine is built from the binary create_pod block (k10s_engine_create_bulk, §8(f)2; the light
cases also take the 4,096 create_node events from the binary K10SNOD1 block) and runs R
seed-perturbed replicas in one batch; each checked replica is replayed by the oracle on its
materialized trace (workloads.replica_scenario).  Counters (incl. attempts, requeued, flushed),
clock, estimator bits + histograms, queue lengths and every placement (pod, node, time bits) must
match.
"""
import pytest

import oracle_jobs
import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd import workloads as wl
from kubernetriks_amd.scenario import SimulationConfig, scenario_bulk


def _engine(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


def _check(backend, cluster, workload, R, checked, base_seed, max_time=1e7, tweak=None, cluster_blob=False):
    cfg = SimulationConfig()
    scn, blob = scenario_bulk(cfg, cluster, workload, cluster_blob=cluster_blob)
    E = _engine(backend)
    probe = E(scn, 1, pods_blob=blob)
    params = wl.replica_params(probe.default_params(), R, base_seed=base_seed, perturb=True)
    if tweak:
        tweak(params)
    del probe
    caps = parity.parity_caps(False)
    eng = E(scn, R, params=params, caps=caps, pods_blob=blob)
    eng.run_until_all_finished(max_time)
    ods = oracle_jobs.replay_many([wl.replica_scenario(cfg, cluster, workload, params[r]) for r in checked], max_time)
    for r, od in zip(checked, ods):
        bad = parity.compare(od, eng, r=r, log=False)
        assert bad == [], (r, bad[:4])
    return [eng.results()[r] for r in checked]


# ---- light load ---------------------------------------------------------------------------------
def test_c3_4096_nodes_host():
    c, w = wl.c3_traces(n_nodes=4096, n_pods=500, arrival_window=40.0, seed=11)
    res = _check("host", c, w, R=2, checked=[0, 1], base_seed=400, cluster_blob=True)
    assert all(x["counters"]["placements"] == 500 for x in res)


@pytest.mark.gpu
def test_c3_4096_nodes_gpu():
    """8 replicas x 4,096 nodes x 4,096 pods (the bench's arrival rate), 4 replayed by the oracle;
    the scenario is built entirely from binary blocks (K10SNOD1 cluster + K10SPOD1 pods)."""
    c, w = wl.c3_traces(n_nodes=4096, n_pods=4096, arrival_window=300.0, seed=2017)
    res = _check("gpu", c, w, R=8, checked=[0, 3, 5, 7], base_seed=123, cluster_blob=True)
    for x in res:
        k = x["counters"]
        assert k["placements"] == k["attempts"] == 4096 and k["nodes_scanned"] == 4096 * 4096
        assert x["status"] == "finished"


# ---- backlog ------------------------------------------------------------------------------------
def _small_backlog(n_pods=5000, window=200.0, duration=600.0):
    # 4,096 nodes, pods of 0.9-1.0 of a modal node's RAM (one per node), arrivals staying long
    # enough that more than 4,096 are wanted at once: hundreds of pods wait at the peak
    return wl.c3_backlog_traces(n_nodes=4096, n_pods=n_pods, arrival_window=window, seed=21, mean_duration=duration,
                                ram_frac=(0.9, 1.0))


def _assert_backlog(k):
    assert k["attempts"] > k["placements"], k
    assert k["requeued"] > 0, k
    assert k["placements"] == k["total_pods_in_trace"]


def test_c3_backlog_4096_nodes_host():
    c, w = _small_backlog(n_pods=4400, window=40.0, duration=150.0)
    res = _check("host", c, w, R=1, checked=[0], base_seed=500)
    _assert_backlog(res[0]["counters"])


@pytest.mark.gpu
def test_c3_backlog_4096_nodes_gpu():
    c, w = _small_backlog()
    res = _check("gpu", c, w, R=8, checked=[0, 2, 5, 7], base_seed=500)
    for x in res:
        _assert_backlog(x["counters"])


@pytest.mark.gpu
def test_c3_backlog_full_size_gpu():
    """The bench's c3_backlog workload itself (16,384 pods), 4 replicas replayed: two with the
    default policy (every pod finish moves the whole unschedulable map back: ~5 attempts per
    placement) and two with enable_unscheduled_pods_conditional_move (scheduler.rs:366-379: pods
    stay until they fit, so the 30-s flush of entries older than 300 s moves them)."""
    c, w = wl.c3_backlog_traces()

    def tweak(params):
        for p in params[2:]:
            p.enable_unscheduled_pods_conditional_move = 1

    res = _check("gpu", c, w, R=4, checked=[0, 1, 2, 3], base_seed=123, tweak=tweak)
    for i, x in enumerate(res):
        k = x["counters"]
        _assert_backlog(k)
        if i < 2:
            assert k["attempts"] > 3 * k["placements"] and k["flushed"] == 0, k
        else:
            assert k["flushed"] > 0, k
            assert x["estimators"]["pod_queue_time"][2] > 300.0  # waited past the flush age


# ---- node churn ---------------------------------------------------------------------------------
def _churn(n_pods, window, removed_frac=0.5, seed=31):
    """C3 cluster where a random half of the nodes is removed while pods run and a quarter of those
    is created again under the same names later, so
    the screened scan meets removed nodes (their cache entries are (0, 0), k10s_engine.h
    S_REMOVE_NODE), pods rescheduled from removed nodes (scheduler.rs:352-364) and re-added nodes."""
    import random
    c, w = wl.c3_traces(n_nodes=4096, n_pods=n_pods, arrival_window=window, seed=seed)
    rng = random.Random(seed)
    nodes = [e.node for e in c.events if e.kind == "create_node"]
    gone = rng.sample(nodes, int(removed_frac * len(nodes)))
    for i, nd in enumerate(gone):
        c.remove_node(window * (0.2 + 0.5 * i / len(gone)), nd.name)
    for nd in gone[: len(gone) // 4]:
        c.create_node(window * 0.8, nd)
    return c, w


def test_c3_node_churn_host():
    c, w = _churn(n_pods=600, window=40.0)
    res = _check("host", c, w, R=1, checked=[0], base_seed=600)
    assert res[0]["counters"]["placements"] >= 600


@pytest.mark.gpu
def test_c3_node_churn_gpu():
    c, w = _churn(n_pods=4096, window=300.0)
    res = _check("gpu", c, w, R=8, checked=[0, 3, 6], base_seed=600, cluster_blob=True)
    for x in res:
        assert x["status"] == "finished" and x["counters"]["placements"] >= 4096, x["counters"]
