"""The exact workloads bench.py measures, oracle-checked: the same traces, the same
bulk scenario path (scenario_bulk + k10s_engine_create_bulk), the same replica count and the same
per-replica parameters (ensemble.shard_params at the bench seed), with bit-exact oracle replays of
replicas spread over the batch (32 by hash, the first and last, and the fewest- and most-event ones).
The replayed batch keeps placement logs and pod records so they can be compared; the batch with
bench.py's own capacities (no logs, the default delay rings, full scans: the exact timed
configuration) runs beside it and must produce the identical counter matrix,
estimators, histograms, clocks and statuses for every replica."""
import pytest

import oracle_jobs
import parity
from kubernetriks_amd import ensemble
from kubernetriks_amd import workloads as wl
from kubernetriks_amd.scenario import SimulationConfig, scenario_bulk

R, NODES, PODS, WINDOW = 8192, 4096, 16384, 1200.0   # bench.py defaults
CHECK = 32   # replicas replayed per batch, chosen by hash across it (+ the edges and the event-count extremes)


def pick(res, k: int):
    """k replicas spread over the batch by a hash of their index, plus the first and last replica and
    the replicas with the fewest and the most delivered events."""
    import hashlib
    n = len(res)
    chosen = sorted(range(n), key=lambda r: hashlib.sha1(f"k10s-replay-{r}".encode()).hexdigest())[:k]
    ev = [x["counters"]["events"] for x in res]
    chosen += [0, n - 1, ev.index(min(ev)), ev.index(max(ev))]
    return sorted(set(chosen))


def _bench_batch(cluster, workload, check, score_plugins=1):
    from kubernetriks_amd.native import Engine
    cfg = SimulationConfig()
    scn, blob = scenario_bulk(cfg, cluster, workload)
    defaults = Engine(scn, 1, pods_blob=blob).default_params()
    params = ensemble.shard_params(defaults, R, 0, base_seed=123, perturb=True)
    for p in params:
        p.score_plugins = score_plugins
        if score_plugins & 2:
            p.most_allocated_weight = 1.0
    caps = parity.parity_caps(False)
    caps.placement_log = PODS + 1024
    eng = Engine(scn, R, params=params, caps=caps, pods_blob=blob)
    eng.run_until_all_finished(1e7)
    res = eng.results()
    # the timed configuration itself: bench.py's Capacities() (pruned_scan 0, delay_fifo 0, no logs)
    from kubernetriks_amd.native import Capacities
    timed = Engine(scn, R, params=params, caps=Capacities(), pods_blob=blob)
    timed.run_until_all_finished(1e7)
    assert (timed.counter_matrix() == eng.counter_matrix()).all()
    tres = timed.results()
    for r in range(R):
        a, b = res[r], tres[r]
        assert (a["status"], a["error_code"], parity.fbits(a["time"])) == \
            (b["status"], b["error_code"], parity.fbits(b["time"])), r
        for k in a["estimators"]:
            ea, eb = a["estimators"][k], b["estimators"][k]
            assert ea[0] == eb[0] and all(parity.feq(x, y) for x, y in zip(ea[1:5], eb[1:5])) and ea[5] == eb[5], (r, k)
    del timed
    if isinstance(check, int):
        check = pick(res, check)
    ods = oracle_jobs.replay_many([wl.replica_scenario(cfg, cluster, workload, params[r]) for r in check], 1e7)
    for r, od in zip(check, ods):
        assert parity.compare(od, eng, r=r, log=False) == [], r
    assert all(x["status"] == "finished" for x in res)
    return res


@pytest.mark.gpu
def test_bench_c3_workload_gpu():
    cluster, workload = wl.c3_traces(NODES, PODS, WINDOW)
    res = _bench_batch(cluster, workload, CHECK)
    assert all(x["counters"]["placements"] == PODS for x in res)


@pytest.mark.gpu
def test_bench_c3_backlog_workload_gpu():
    cluster, workload = wl.c3_backlog_traces(NODES, PODS, WINDOW)
    res = _bench_batch(cluster, workload, CHECK)
    # the regime it is there for: failed attempts and unschedulable-map traffic in every replica
    assert all(x["counters"]["attempts"] > x["counters"]["placements"] for x in res)


@pytest.mark.gpu
def test_bench_c3_most_allocated_gpu():
    """bench.py --score-plugins both (LeastAllocated + MostAllocated, weights 1 and 1)."""
    cluster, workload = wl.c3_traces(NODES, PODS, WINDOW)
    _bench_batch(cluster, workload, [0, 8191], score_plugins=3)
