"""Per-block Pareto fronts of the packed node cache (k10s_engine.h fr_block / fr_refresh / front_scan,
K10S_FRONT=1): the serial cycle's fast-path attempts (weight 1, rc > 0, rr > 0) score
only each 64-node block's index-aware front — the nodes no later node of the block dominates in both
free cpu and free ram — K10S_FR_K = 8 slots per block, a block with a larger front read whole.

* CPU: a model of the fronts (block front, 8 slots, overflow blocks read whole) picks the
  reference's argmax (kube_scheduler.rs:140-148: Fit, LeastAllocated, last maximum) on adversarial
  node sets, including fronts of exactly 8, 9 and 64 nodes per block and ragged last blocks.
* Host and GPU: clusters built so the fronts overflow (staircases), sit at the slot count, tie
  (identical nodes), end in a ragged block, and lose and regain nodes mid-run, through the event loop
  against the oracle event for event; the host run checks the fronts cut the entries read, and that
  a cache over 4,096 nodes or up to 512 (fronts off) reads every node per attempt; random scenarios
  over 520-1,119 nodes.
"""
import os
import random

import pytest

import gen
import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd.scenario import GenericClusterTrace, GenericWorkloadTrace, Node, Pod, SimulationConfig, scenario_text
from test_scan_adversarial import la, reference_argmax

K = 8   # K10S_FR_K


def block_front(cpu, ram, lo, hi):
    """Block [lo, hi)'s index-aware front, ascending: kept iff no kept later node dominates it."""
    kept = []
    for n in range(hi - 1, lo - 1, -1):
        if cpu[n] == 0 and ram[n] == 0:
            continue   # an absent node holds (0, 0)
        if not any(cpu[m] >= cpu[n] and ram[m] >= ram[n] for m in kept):
            kept.append(n)
    return kept[::-1]


def front_argmax(cpu, ram, rc, rr, stats=None):
    """The fronts' scan: every block's first K front nodes, plus the whole block when its front is
    larger; the (score, index) maximum of the fitting candidates."""
    N = len(cpu)
    cand = []
    for lo in range(0, N, 64):
        hi = min(lo + 64, N)
        fr = block_front(cpu, ram, lo, hi)
        cand += fr[:K]
        if len(fr) > K:
            cand += range(lo, hi)
            if stats is not None:
                stats["over"] = stats.get("over", 0) + 1
    best = None
    for n in cand:
        if rc <= cpu[n] and rr <= ram[n]:
            k = (la(cpu[n], ram[n], rc, rr), n)
            if best is None or k > best:
                best = k
    return best[1] if best else -1


def staircase(N, rng, length=64, base_c=60000, base_r=1 << 37):
    """Blocks whose last `length` nodes trade cpu for ram (each later node: more cpu, less ram), so
    the front is exactly those nodes; the nodes before them are dominated."""
    cpu, ram = [], []
    for b in range(0, N, 64):
        m = min(64, N - b)
        off = rng.randint(0, 4000)
        for i in range(m):
            j = i - (m - length)
            if j < 0:
                cpu.append(rng.randint(1000, base_c // 2)), ram.append(rng.randint(1 << 30, base_r >> 2))
            else:
                cpu.append(base_c + off + 37 * j), ram.append(base_r - (1 << 24) * j - off)
    return cpu, ram


def node_sets(N, seed):
    rng = random.Random(seed)
    out = {}
    out["staircase64"] = staircase(N, rng, 64)
    out["front8"] = staircase(N, rng, 8)
    out["front9"] = staircase(N, rng, 9)
    out["front17"] = staircase(N, rng, 17)
    # C3-like: identical empty nodes (ties), a few big ones, partly used ones
    cpu, ram = [], []
    for _ in range(N):
        k = rng.choice([0, 0, 0, 1, 2])
        big = rng.random() < 0.03
        cpu.append(64000 - 500 * k + (32000 if big else 0))
        ram.append(int((1.5 if big else 1.0) * 0.69 * (1 << 37)) - k * (1 << 29))
    out["c3_like"] = (cpu, ram)
    # descending free ram at equal cpu: every node its block's front (cpu ties, ram falls)
    out["descending"] = ([64000] * N, [(1 << 38) - (1 << 20) * n for n in range(N)])
    return out


def test_front_model_picks_the_reference_argmax():
    stats = {}
    for seed in range(3):
        for N in (64, 65, 511, 1000):
            for name, (cpu, ram) in node_sets(N, seed).items():
                rng = random.Random(seed * 7 + N)
                for _ in range(6):
                    rc = rng.choice([1, 500, 1000, 30000, 70000])
                    rr = rng.choice([1, 1 << 20, 1 << 30, 1 << 36, 1 << 38])
                    want = reference_argmax(cpu, ram, [True] * N, rc, rr)
                    assert front_argmax(cpu, ram, rc, rr, stats) == want, (seed, N, name, rc, rr)
    assert stats["over"] > 0


def test_block_front_sizes():
    rng = random.Random(3)
    for length in (1, 8, 9, 17, 64):
        cpu, ram = staircase(256, rng, length)
        for lo in range(0, 256, 64):
            assert len(block_front(cpu, ram, lo, lo + 64)) == length, length


def _scenario(cpu, ram, n_pods, seed, churn=False):
    """The node set as a cluster at t=0, a pod stream of small requests (20 per second); with churn,
    nodes of every block leave at t=3 and come back (new names, same capacities) at t=6."""
    rng = random.Random(seed)
    c = GenericClusterTrace()
    for i, (a, r) in enumerate(zip(cpu, ram)):
        c.create_node(0.0, Node(f"node_{i:05d}", max(int(a), 1), max(int(r), 1)))
    if churn:
        for i in range(5, len(cpu), 23):
            c.remove_node(3.0, f"node_{i:05d}")
            c.create_node(6.0, Node(f"node_b{i:05d}", max(int(cpu[i]), 1), max(int(ram[i]), 1)))
    w = GenericWorkloadTrace()
    for i in range(n_pods):
        w.create_pod(float(1 + i // 20), Pod(f"pod_{i:05d}", rng.choice([1, 500, 1000, 3000]),
                                             rng.choice([1, 1 << 20, 1 << 28, 1 << 30, 3 << 30]),
                                             float(rng.randint(50, 400))))
    return scenario_text(SimulationConfig(), c, w)


def _engine(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


BACKENDS = ["host", pytest.param("gpu", marks=pytest.mark.gpu)]
KINDS = ["staircase64", "front8", "front9", "front17", "c3_like", "descending"]


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("kind", KINDS)
def test_front_clusters_in_the_event_loop(backend, kind):
    N = 4096 if backend == "gpu" else 640
    cpu, ram = node_sets(N, 11)[kind]
    scn = _scenario(cpu, ram, 400 if backend == "gpu" else 160, seed=len(kind))
    od, eng = parity.run_pair(_engine(backend), scn, max_time=50000.0)
    assert parity.compare(od, eng) == [], kind


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("N", [4000, 4033, 4095])
def test_front_ragged_last_block(backend, N):
    if backend == "host":
        N = 513 + N % 100   # 513, 546, 608: ragged, and above the 512 nodes below which fronts are off
    cpu, ram = node_sets(N, 5)["front9"]
    scn = _scenario(cpu, ram, 300 if backend == "gpu" else 120, seed=N)
    od, eng = parity.run_pair(_engine(backend), scn, max_time=50000.0)
    assert parity.compare(od, eng) == [], N


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("kind", ["staircase64", "c3_like"])
def test_front_node_removal_and_return(backend, kind):
    """Removed nodes' entries drop to (0, 0) and their blocks rebuild; returning nodes land at new
    cache positions (new names sort after the old ones) and rebuild theirs."""
    N = 2048 if backend == "gpu" else 576
    cpu, ram = node_sets(N, 13)[kind]
    scn = _scenario(cpu, ram, 300 if backend == "gpu" else 140, seed=3, churn=True)
    od, eng = parity.run_pair(_engine(backend), scn, max_time=50000.0)
    assert parity.compare(od, eng) == [], kind
    assert eng.results()[0]["counters"]["processed_nodes"] > N


def test_fronts_read_fewer_entries_host():
    """c3_like at 1,024 nodes: the fronts read a fraction of the cache per attempt; the same cluster
    over 4,096 nodes of capacity (one extra node: 4,097, no fronts) reads it all, and so does one of
    512 nodes (fronts only above 512)."""
    rng = random.Random(1)
    cpu, ram = node_sets(1024, 2)["c3_like"]
    scn = _scenario(cpu, ram, 200, seed=9)
    od, eng = parity.run_pair(HostEngine, scn, max_time=50000.0, log=False)
    assert parity.compare(od, eng, log=False) == []
    k = eng.results()[0]["counters"]
    assert k["attempts"] >= 200 and k["nodes_read"] < 0.35 * 1024 * k["attempts"], k
    cpu2 = cpu * 4 + [rng.randint(1000, 60000)]
    ram2 = ram * 4 + [1 << 30]
    scn2 = _scenario(cpu2, ram2, 60, seed=9)
    od2, eng2 = parity.run_pair(HostEngine, scn2, max_time=50000.0, log=False)
    assert parity.compare(od2, eng2, log=False) == []
    k2 = eng2.results()[0]["counters"]
    assert k2["nodes_read"] >= 4097 * k2["attempts"], k2
    # up to 512 nodes a full scan is one memory round trip: no fronts (k10s_builder.cpp make_layout)
    scn3 = _scenario(cpu[:512], ram[:512], 60, seed=9)
    od3, eng3 = parity.run_pair(HostEngine, scn3, max_time=50000.0, log=False)
    assert parity.compare(od3, eng3, log=False) == []
    k3 = eng3.results()[0]["counters"]
    assert k3["nodes_read"] >= 512 * k3["attempts"], k3


# Random scenarios (tests/gen.py: mixed node sizes, removals, default groups, integer and real
# times, conditional move) over 520-1,119 nodes, so the fronts are on.  K10S_FRONT_FUZZ_GPU_SEEDS=N
# widens the GPU sweep.
FRONT_FUZZ_GPU = list(range(int(os.environ.get("K10S_FRONT_FUZZ_GPU_SEEDS", "24"))))


def _front_fuzz(backend, seed):
    scn = gen.random_scenario(50_000 + seed, n_pods=300, n_nodes=520 + (seed * 37) % 600)
    od, eng = parity.run_pair(_engine(backend), scn, max_time=20000.0)
    assert parity.compare(od, eng) == [], seed


@pytest.mark.parametrize("seed", range(4))
def test_front_fuzz_host(seed):
    _front_fuzz("host", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", FRONT_FUZZ_GPU)
def test_front_fuzz_gpu(seed):
    _front_fuzz("gpu", seed)


@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("kind", ["staircase64", "front9", "c3_like"])
def test_front_invariant_between_events(backend, kind):
    """White-box: at checkpoints through a run (launches of 13 events), every block not marked stale
    holds exactly its index-aware front in its slots and the right overflow bit, recomputed from the
    replica's node cache (k10s_engine_check_fronts; the host engine's hc_check_fronts); the run still
    equals the oracle."""
    N = 2048 if backend == "gpu" else 640
    cpu, ram = node_sets(N, 23)[kind]
    scn = _scenario(cpu, ram, 300 if backend == "gpu" else 160, seed=5, churn=True)
    eng = _engine(backend)(scn, 2, caps=parity.parity_caps(True, gauges=parity.GAUGE_ROWS))
    checked = 0
    for t in range(1, 400, 7):
        eng.step_until_time(float(t), 13)
        checked += eng.check_fronts(0) + eng.check_fronts(1)
    assert checked > 0
    eng.run_until_all_finished(50000.0)
    od, _ = parity.run_pair(HostEngine, scn, max_time=50000.0)
    assert parity.compare(od, eng) == [], kind
