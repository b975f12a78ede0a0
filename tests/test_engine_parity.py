"""Engine vs oracle parity: bit-exact counters, estimators, clocks, placements, per-pod times and
per-event (id, time, kind, pod, node, slot) logs.

Each test body runs against two backends:
  * "gpu"  — the product: build/libk10s.so on a MI355X (pytest -m gpu);
  * "host" — the TEST-ONLY host build of the same engine source (tests/hostcheck), on CPU.
"""
import os
import math
import random

import pytest

import gen
import oracle_bridge as ob
import parity
import scenarios as sc
from hostcheck_bridge import HostEngine
from kubernetriks_amd import workloads as wl
from kubernetriks_amd.native import RUN_UNTIL_ALL_FINISHED, RUN_UNTIL_TIME
from kubernetriks_amd.scenario import SimulationConfig, scenario_text


def _gpu_engine():
    from kubernetriks_amd.native import Engine
    return Engine


BACKENDS = [
    pytest.param("host", id="host"),
    pytest.param("gpu", id="gpu", marks=pytest.mark.gpu),
]


def engine_cls(backend):
    return HostEngine if backend == "host" else _gpu_engine()


STEP_SCENARIOS = {"node_removed_same_time_as_assignment": 1000.0, "hpa": 1200.0}


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("name", sorted(sc.ALL_TEST_SCENARIOS))
def test_reference_scenarios(backend, name):
    scn = sc.ALL_TEST_SCENARIOS[name]()
    if name in STEP_SCENARIOS:
        od, eng = parity.run_pair(engine_cls(backend), scn, mode=RUN_UNTIL_TIME, until=STEP_SCENARIOS[name])
    else:
        od, eng = parity.run_pair(engine_cls(backend), scn)
    assert parity.compare(od, eng) == []


@pytest.mark.parametrize("backend", BACKENDS)
def test_hpa_checkpoints(backend):
    """tests/test_hpa.rs:91-134 through the engine's stepping API."""
    import json, os
    G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.json")))
    eng = engine_cls(backend)(sc.sc_hpa(), 1, caps=parity.parity_caps(False))
    for t, size in G["hpa"]["checkpoints"]:
        eng.step_until_time(t)
        assert eng.group_sizes(0)["pod_group_1"][0] == size, t


FUZZ_SEEDS_HOST = list(range(0, 240))
# K10S_FUZZ_GPU_SEEDS=N widens the GPU sweep to seeds 0..N-1 (an extended run, e.g. after kernel
# changes; the default keeps the round-end suite short)
FUZZ_SEEDS_GPU = list(range(0, int(os.environ.get("K10S_FUZZ_GPU_SEEDS", "60"))))


def _fuzz(backend, seed):
    kw = dict(ca=(seed % 3 == 1), hpa=(seed % 4 == 2))
    scn = gen.random_scenario(seed, **kw)
    mode = RUN_UNTIL_TIME if kw["hpa"] else RUN_UNTIL_ALL_FINISHED
    od, eng = parity.run_pair(engine_cls(backend), scn, mode=mode, until=3000.0, max_time=20000.0)
    assert parity.compare(od, eng) == [], seed


@pytest.mark.parametrize("seed", FUZZ_SEEDS_HOST)
def test_fuzz_host(seed):
    _fuzz("host", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", FUZZ_SEEDS_GPU)
def test_fuzz_gpu(seed):
    _fuzz("gpu", seed)


# Wide random scenarios: 50-200 nodes (node caches of one to four 64-lane scan steps, where the
# small sweep above never leaves the first step) and 200-800 pods over a 1,200 s horizon, with and
# without removals.  K10S_FUZZ_WIDE_GPU_SEEDS=N widens the GPU sweep.
FUZZ_WIDE_HOST = list(range(10_000, 10_024))
FUZZ_WIDE_GPU = list(range(10_000, 10_000 + int(os.environ.get("K10S_FUZZ_WIDE_GPU_SEEDS", "24"))))


def _fuzz_wide(backend, seed):
    rng = random.Random(seed)
    kw = dict(ca=(seed % 3 == 1), hpa=(seed % 4 == 2), removals=(seed % 2 == 0))
    scn = gen.random_scenario(seed, n_pods=rng.choice([200, 400, 800]), n_nodes=rng.randint(50, 200),
                              horizon=1200.0, **kw)
    mode = RUN_UNTIL_TIME if kw["hpa"] else RUN_UNTIL_ALL_FINISHED
    od, eng = parity.run_pair(engine_cls(backend), scn, mode=mode, until=3000.0, max_time=20000.0)
    assert parity.compare(od, eng) == [], seed


@pytest.mark.parametrize("seed", FUZZ_WIDE_HOST)
def test_fuzz_wide_host(seed):
    _fuzz_wide("host", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", FUZZ_WIDE_GPU)
def test_fuzz_wide_gpu(seed):
    _fuzz_wide("gpu", seed)


# Delay-class FIFO rings are an optimisation of the event queue: tiny rings (constant spill to the
# heap), one-entry rings and no rings at all must deliver the identical event sequence.
FIFO_CASES = [(seed, fifo) for seed in (1, 4, 6, 10, 13, 22) for fifo in (1, 2, 0xFFFFFFFF)]


@pytest.mark.parametrize("seed,fifo", FIFO_CASES)
def test_fifo_capacity_host(seed, fifo):
    kw = dict(ca=(seed % 3 == 1), hpa=(seed % 4 == 2))
    mode = RUN_UNTIL_TIME if kw["hpa"] else RUN_UNTIL_ALL_FINISHED
    od, eng = parity.run_pair(engine_cls("host"), gen.random_scenario(seed, **kw), mode=mode, until=3000.0,
                              max_time=20000.0, fifo=fifo)
    assert parity.compare(od, eng) == [], (seed, fifo)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,fifo", FIFO_CASES)
def test_fifo_capacity_gpu(seed, fifo):
    kw = dict(ca=(seed % 3 == 1), hpa=(seed % 4 == 2))
    mode = RUN_UNTIL_TIME if kw["hpa"] else RUN_UNTIL_ALL_FINISHED
    od, eng = parity.run_pair(engine_cls("gpu"), gen.random_scenario(seed, **kw), mode=mode, until=3000.0,
                              max_time=20000.0, fifo=fifo)
    assert parity.compare(od, eng) == [], (seed, fifo)


# Block-bound pruned scan: many-node clusters (several 64-node blocks), identical
# nodes (score ties decided by the last index), node removals; the pruned engine, the full-scan
# engine and the oracle must agree event for event.
PRUNE_SEEDS = list(range(200, 216))


def _prune_case(backend, seed, pruned):
    n_nodes = (70, 130, 257, 400)[seed % 4]
    scn = gen.random_scenario(seed, n_pods=240, n_nodes=n_nodes, same_nodes=(seed % 2 == 0))
    od, eng = parity.run_pair(engine_cls(backend), scn, max_time=40000.0, pruned=pruned)
    assert parity.compare(od, eng) == [], (seed, pruned)
    return eng.results()[0]["counters"]


@pytest.mark.parametrize("seed", PRUNE_SEEDS)
def test_pruned_scan_many_nodes_host(seed):
    c = _prune_case("host", seed, 1)
    f = _prune_case("host", seed, 0)
    assert c["placements"] == f["placements"] and c["attempts"] == f["attempts"]


def test_pruned_scan_reads_less():
    """The bound prunes where blocks differ: big nodes first in name order, small ones after."""
    from kubernetriks_amd.scenario import GenericClusterTrace, GenericWorkloadTrace, Node, Pod
    c = GenericClusterTrace()
    for i in range(256):
        big = i < 64
        c.create_node(0.0, Node(f"node_{i:03d}", 128000 if big else 8000, (256 if big else 16) << 30))
    w = GenericWorkloadTrace()
    for i in range(300):
        w.create_pod(float(1 + i // 10), Pod(f"pod_{i:03d}", 500 + (i % 7) * 100, (1 + i % 3) << 30, 400.0))
    scn = scenario_text(SimulationConfig(), c, w)
    od, eng = parity.run_pair(engine_cls("host"), scn, max_time=1e6, pruned=1)
    assert parity.compare(od, eng) == []
    k = eng.results()[0]["counters"]
    # each node addition re-derives its block's bound (64 entries); the rest is scans + upkeep
    per_attempt = (k["nodes_read"] - 64 * k["processed_nodes"]) / k["attempts"]
    assert k["attempts"] == 300 and per_attempt < 0.8 * 256, k


@pytest.mark.gpu
@pytest.mark.parametrize("seed", PRUNE_SEEDS)
def test_pruned_scan_many_nodes_gpu(seed):
    c = _prune_case("gpu", seed, 1)
    f = _prune_case("gpu", seed, 0)
    assert c["placements"] == f["placements"] and c["attempts"] == f["attempts"]


@pytest.mark.parametrize("backend", BACKENDS)
def test_budgeted_launches_equal_one_launch(backend):
    """Pausing every few events (multi-launch runs) must not change anything."""
    scn = gen.random_scenario(7, n_pods=80)
    E = engine_cls(backend)
    a = E(scn, 1, caps=parity.parity_caps(True))
    a.run_until_all_finished(20000.0)
    b = E(scn, 1, caps=parity.parity_caps(True))
    b.run_until_all_finished(20000.0, max_events_per_launch=37)
    assert a.results() == b.results()
    assert a.event_log(0) == b.event_log(0)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("seed,budget", [(10_001, 37), (10_004, 101), (10_007, 1), (10_010, 513)])
def test_budgeted_wide_scenarios_match_oracle(backend, seed, budget):
    """Wide random scenarios (_fuzz_wide's shapes, without HPA) paused every `budget` events, each
    resumed launch re-reading the replica from HBM, against the oracle's single run."""
    rng = random.Random(seed)
    scn = gen.random_scenario(seed, n_pods=rng.choice([200, 400, 800]), n_nodes=rng.randint(50, 200),
                              horizon=1200.0, ca=(seed % 3 == 1), removals=(seed % 2 == 0))
    od, eng = parity.run_pair(engine_cls(backend), scn, max_time=20000.0, budget=budget)
    assert parity.compare(od, eng) == [], (seed, budget)


@pytest.mark.parametrize("backend", BACKENDS)
def test_batched_replicas_match_oracle_per_replica(backend):
    """R seed-perturbed replicas in one batch: each equals the oracle on its materialized trace."""
    c, w = wl.c3_traces(n_nodes=256, n_pods=600, arrival_window=300.0, seed=5)
    cfg = SimulationConfig()
    scn = scenario_text(cfg, c, w)
    E = engine_cls(backend)
    R = 48 if backend == "gpu" else 6
    probe = E(scn, 1)
    params = wl.replica_params(probe.default_params(), R, base_seed=1000, perturb=True)
    eng = E(scn, R, params=params, caps=parity.parity_caps(False))
    eng.run_until_all_finished(1e6)
    for r in sorted({0, R // 2, R - 1}):
        o = ob.OracleSim(scenario_text(cfg, c, wl.perturb_workload(w, params[r].seed)))
        st = o.run_until_all_finished(1e6)
        od = o.result(placements=True)
        od["status_name"] = parity.ORACLE_STATUS[st]
        assert parity.compare(od, eng, r=r, log=False) == [], r


# ---- unit-parity surface: k10s_schedule_one_batch ---------------------------------------------
def _random_problem(rng, n_nodes):
    nodes = []
    for i in range(n_nodes):
        if rng.random() < 0.1:
            cpu = 0
        else:
            cpu = rng.choice([1000, 2000, 4000, 8000, rng.randint(1, 20000)])
        ram = rng.choice([0, 1 << 30, 2 << 30, 4 << 30, rng.randint(1, 1 << 34)]) if rng.random() < 0.9 else 0
        present = rng.random() < 0.85
        nodes.append((f"n{i:05d}", cpu, ram, present))
    r = rng.random()
    if r < 0.05:
        pc, pr = 0, 0
    elif r < 0.15:
        pc, pr = 0, rng.randint(1, 1 << 30)
    else:
        pc, pr = rng.choice([500, 1000, 2000]), rng.choice([1 << 28, 1 << 30])
    return nodes, pc, pr


@pytest.mark.gpu
def test_schedule_one_batch_matches_oracle():
    import ctypes
    import torch
    from kubernetriks_amd.native import lib
    rng = random.Random(11)
    R, N, stride = 400, 300, 320
    cpu = torch.zeros(R * stride, dtype=torch.int64)
    ram = torch.zeros(R * stride, dtype=torch.int64)
    bits = torch.zeros(R * stride // 64, dtype=torch.int64)
    rc = torch.zeros(R, dtype=torch.int64)
    rr = torch.zeros(R, dtype=torch.int64)
    problems = []
    for r in range(R):
        nodes, pc, pr = _random_problem(rng, N if r % 7 else rng.randint(0, 5))
        problems.append((nodes, pc, pr))
        for i, (_, c_, r_, p_) in enumerate(nodes):
            cpu[r * stride + i] = c_
            ram[r * stride + i] = r_ - (1 << 64) if r_ >= (1 << 63) else r_
            if p_:
                w = (r * stride + i) // 64
                v = int(bits[w]) & ((1 << 64) - 1)
                v |= 1 << ((r * stride + i) % 64)
                bits[w] = v - (1 << 64) if v >= (1 << 63) else v
        rc[r], rr[r] = pc, pr
    dev = torch.device("cuda:0")
    d_cpu = cpu.to(torch.int32).to(dev)
    d_ram, d_bits = ram.to(dev), bits.to(dev)
    d_rc, d_rr = rc.to(torch.int32).to(dev), rr.to(dev)
    out_node = torch.full((R,), -7, dtype=torch.int32, device=dev)
    out_st = torch.full((R,), -7, dtype=torch.int32, device=dev)
    rcode = lib().k10s_schedule_one_batch(d_cpu.data_ptr(), d_ram.data_ptr(), d_bits.data_ptr(), N, stride,
                                          d_rc.data_ptr(), d_rr.data_ptr(), 1.0, R, out_node.data_ptr(),
                                          out_st.data_ptr(), None)
    assert rcode == 0
    torch.cuda.synchronize()
    got_n, got_s = out_node.cpu().tolist(), out_st.cpu().tolist()
    for r, (nodes, pc, pr) in enumerate(problems):
        present = [(nm, c_, r_) for nm, c_, r_, p_ in nodes if p_]
        st, name = ob.schedule_one(present, pc, pr)
        assert got_s[r] == st, r
        if st == 0:
            assert nodes[got_n[r]][0] == name, r


@pytest.mark.gpu
def test_host_buffer_scheduler_matches_oracle():
    """k10s_scheduler_schedule (host arrays, the Rust adapter's surface) vs the oracle."""
    import numpy as np
    from kubernetriks_amd.native import Scheduler
    rng = random.Random(23)
    R, N = 257, 130
    cpu = np.zeros((R, N), np.uint32)
    ram = np.zeros((R, N), np.uint64)
    bits = np.zeros((R, (N + 63) // 64), np.uint64)
    rc = np.zeros(R, np.uint32)
    rr = np.zeros(R, np.uint64)
    problems = []
    for r in range(R):
        nodes, pc, pr = _random_problem(rng, N if r % 5 else rng.randint(0, 3))
        problems.append((nodes, pc, pr))
        for i, (_, c_, r_, p_) in enumerate(nodes):
            cpu[r, i], ram[r, i] = c_, r_
            if p_:
                bits[r, i // 64] |= np.uint64(1 << (i % 64))
        rc[r], rr[r] = pc, pr
    s = Scheduler(N, R)
    got_n, got_s = s.schedule(cpu, ram, rc, rr, bits)
    for r, (nodes, pc, pr) in enumerate(problems):
        present = [(nm, c_, r_) for nm, c_, r_, p_ in nodes if p_]
        st, name = ob.schedule_one(present, pc, pr)
        assert got_s[r] == st, r
        if st == 0:
            assert nodes[got_n[r]][0] == name, r
    # present_bits=None: every node in the cache
    nodes, pc, pr = problems[1]
    n1, s1 = s.schedule(cpu[1:2], ram[1:2], rc[1:2], rr[1:2], None)
    st, name = ob.schedule_one([(nm, c_, r_) for nm, c_, r_, _ in nodes], pc, pr)
    assert s1[0] == st and (st != 0 or nodes[n1[0]][0] == name)
    s.close()


# ---- ScorePlugin surface: k10s_score_batch, bit for bit ----------------------------------------
def _score_inputs(n, seed):
    """(alloc_cpu u32, alloc_ram u64, req_cpu u32, req_ram u64): random pairs over the whole operand
    ranges (ram log-uniform up to 2^64 - 1, so u64 -> f64 rounding is exercised), plus edge rows:
    alloc == req (0 quotient), 0/0 (NaN), 2^53 +- 1, 2^64 - 1, powers of two."""
    import numpy as np
    g = np.random.default_rng(seed)
    ac = g.integers(1, 1 << 32, n, dtype=np.uint64)
    ac[: n // 4] = g.integers(1, 1 << 17, n // 4)                      # kube-sized millicores
    rc = (ac.astype(np.float64) * g.random(n)).astype(np.uint64)
    bits = g.integers(1, 65, n)
    ar = g.integers(0, 1 << 64, n, dtype=np.uint64, endpoint=False) >> (64 - bits).astype(np.uint64)
    ar = np.maximum(ar, np.uint64(1))
    rr = np.minimum((ar.astype(np.float64) * g.random(n)).astype(np.uint64), ar)
    edge_c = [0, 0, 1, 64000, 64000, (1 << 32) - 1, (1 << 32) - 1, 2, 3]
    edge_rc = [0, 0, 1, 64000, 500, 0, (1 << 32) - 1, 1, 1]
    edge_r = [0, 5, 1, (1 << 53) + 1, (1 << 53) - 1, (1 << 64) - 1, (1 << 64) - 1, 1 << 63, 3]
    edge_rr = [0, 5, 0, 1, (1 << 53) - 2, 1, (1 << 64) - 2, 1, 2]
    k = len(edge_c)
    ac[:k], rc[:k], ar[:k], rr[:k] = edge_c, edge_rc, edge_r, edge_rr
    rc = np.minimum(rc, ac)
    return ac.astype(np.uint32), ar, rc.astype(np.uint32), rr


def _score_expected(ac, ar, rc, rr, w):
    """plugin.rs:52-63 with IEEE f64 (numpy: correctly rounded u64 -> f64 and division), then
    0.0 + s * w (kube_scheduler.rs:113-138)."""
    import numpy as np
    with np.errstate(invalid="ignore", divide="ignore"):
        cs = (ac - rc).astype(np.float64) * 100.0 / ac.astype(np.float64)
        rs = (ar - rr).astype(np.float64) * 100.0 / ar.astype(np.float64)
        return 0.0 + ((cs + rs) / 2.0) * w


def test_score_expected_matches_oracle():
    """The numpy restatement used by the GPU test equals the oracle's LeastAllocated, bit for bit."""
    import numpy as np
    ac, ar, rc, rr = _score_inputs(3000, 5)
    exp = _score_expected(ac, ar, rc, rr, 1.0)
    for i in range(len(ac)):
        o = ob.least_allocated(int(ac[i]), int(ar[i]), int(rc[i]), int(rr[i]))
        e = float(exp[i])
        assert (math.isnan(o) and math.isnan(e)) or np.float64(o).view(np.uint64) == np.float64(e).view(np.uint64), i


@pytest.mark.gpu
@pytest.mark.parametrize("weight", [1.0, 0.37, -2.5])
def test_score_batch_bit_exact(weight):
    """The device score (rcp + Newton quotient without div_scale/div_fixup, fma u64 -> f64) equals
    IEEE f64 division bit for bit over 2^21 random pairs and the edge rows."""
    import numpy as np
    import torch
    from kubernetriks_amd.native import lib
    ac, ar, rc, rr = _score_inputs(1 << 21, int(weight * 100) & 0xffff)
    exp = _score_expected(ac, ar, rc, rr, weight)
    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(dev)  # noqa: E731
    d_ac, d_rc = t(ac, np.int32), t(rc, np.int32)
    d_ar, d_rr = t(ar, np.int64), t(rr, np.int64)
    out = torch.empty(len(ac), dtype=torch.float64, device=dev)
    assert lib().k10s_score_batch(d_ac.data_ptr(), d_ar.data_ptr(), d_rc.data_ptr(), d_rr.data_ptr(), weight,
                                  len(ac), out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    nan_g, nan_e = np.isnan(got), np.isnan(exp)
    assert (nan_g == nan_e).all()
    assert nan_e[0] and nan_e.sum() >= 1
    bad = np.nonzero(got[~nan_e].view(np.uint64) != exp[~nan_e].view(np.uint64))[0]
    assert bad.size == 0, (bad[:5], got[~nan_e][bad[:5]], exp[~nan_e][bad[:5]])


# ---- binary create_pod block (k10s_engine_create_bulk) --------------------------
def _bulk_pair(engine_cls, **kw):
    from kubernetriks_amd.scenario import scenario_bulk
    cfg = SimulationConfig()
    c, w = wl.c3_traces(n_nodes=48, n_pods=400, arrival_window=120.0, seed=5)
    text = scenario_text(cfg, c, w)
    btext, blob = scenario_bulk(cfg, c, w)
    assert "create_pod " not in btext and blob[:8] == b"K10SPOD1"
    R = 3
    caps = parity.parity_caps(log=True)
    a = engine_cls(text, R, caps=caps, **kw)
    b = engine_cls(btext, R, caps=caps, pods_blob=blob, **kw)
    for e in (a, b):
        e.run_until_all_finished(1e7)
    for r in range(R):
        assert a.results()[r] == b.results()[r] or repr(a.results()[r]) == repr(b.results()[r]), r
        assert a.placements(r) == b.placements(r)
        assert a.event_log(r) == b.event_log(r)
    assert a.results()[0]["counters"]["placements"] == 400
    return a, b


def test_bulk_pod_blob_equals_text_host():
    _bulk_pair(HostEngine)


def test_bulk_pod_blob_rejects_malformed():
    from kubernetriks_amd.scenario import scenario_bulk
    cfg = SimulationConfig()
    c, w = wl.c3_traces(n_nodes=4, n_pods=10, arrival_window=10.0, seed=1)
    btext, blob = scenario_bulk(cfg, c, w)
    for bad in (blob[:-3], b"K10SPODX" + blob[8:], blob[:16]):
        with pytest.raises(ValueError):
            HostEngine(btext, 1, pods_blob=bad)


@pytest.mark.gpu
def test_bulk_pod_blob_equals_text_gpu():
    from kubernetriks_amd.native import Engine
    _bulk_pair(Engine)


def test_counter_matrix_view_equals_results():
    """bench.py sums counters through EngineBase.counter_matrix (a numpy view of the results array)."""
    from kubernetriks_amd.native import COUNTER_NAMES
    scn = gen.random_scenario(5, n_pods=40)
    e = HostEngine(scn, 3)
    e.run_until_all_finished(20000.0)
    m = e.counter_matrix()
    assert m.shape == (3, len(COUNTER_NAMES))
    for r, res in enumerate(e.results()):
        assert [int(x) for x in m[r]] == [res["counters"][k] for k in COUNTER_NAMES]
