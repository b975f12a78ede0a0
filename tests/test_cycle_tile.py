"""The scheduling cycle's tiles (k10s_engine.h tile_best_pass / run_scheduling_cycle_tiles): after a
cycle with a failed attempt, the cycle pops K10S_TILE (32) pods at a time and reads the packed node
cache once for all of them.  The read finds, per pod and per lane share of the nodes, the best fitting
node of the cache as it is then.  Pods that fit nowhere fail without a scan (exact: nothing is pushed
onto the action queue during a cycle, scheduler.rs:261-330, and a reservation only lowers a node's
allocatable, 118-123).  The others are placed in order from the lane bests, and only the lanes whose
share holds a node reserved earlier in the tile rescan their share (the proof is in the kernel's
comment).

Adversarial cases against the oracle, bit for bit (counters, clock, estimators, every placement and
the whole event log), on the host build and the GPU:
* every pod wants the same node (identical nodes, identical pods, ties to the last index);
* pods that fit nowhere mixed with pods that fit, and tiles in which only later pods fit after
  earlier ones took the room;
* cycles of fewer than, exactly and more than 8 pods (a tile never spans two cycles);
* node removal and re-creation between cycles;
* a removed pod inside a tile (skipped like the loop's `continue`);
* weight != 1, and zero requests, which stay on the serial path; pods with one zero request, which
  the scan places inside a tile;
* the conditional move (pods stay unschedulable) and move-all;
* hundreds of nodes, so lane shares span several 256-node steps, with a ragged last step, and
  identical nodes whose ties span every lane.
Backlog cases also check that the tiles replaced scans (nodes_read)."""
import os
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
                     huge_every: int = 0, pod_removals: bool = False, bursts: bool = True, half_zero_every: int = 0,
                     tiny_every: int = 0) -> str:
    rng = random.Random(seed)
    cfg = SimulationConfig()
    cfg.enable_unscheduled_pods_conditional_move = cond_move
    cfg.scheduling_cycle_interval = cycle
    cfg.score_weight = weight
    c = GenericClusterTrace()
    for k in range(n_nodes):
        cpu = 8000 if identical else rng.choice([4000, 8000, 16000])
        ram = 32 * GIB if identical else rng.choice([16, 32, 64]) * GIB
        if tiny_every and k % tiny_every:   # most nodes hold no pod: a large cache that saturates early
            cpu, ram = 100, GIB // 4
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
        if half_zero_every and i % half_zero_every == 2:
            cpu = 0   # placed by the scan inside a tile (one request > 0): it changes the cache too
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
    "many_nodes": dict(seed=13, n_nodes=700, n_pods=3000),
    "identical_many": dict(seed=14, n_nodes=300, n_pods=2000, identical=True),
    "ragged_520": dict(seed=15, n_nodes=520, n_pods=2500, bursts=False, cycle=5.0),
    "identical_cond_move_many": dict(seed=16, n_nodes=260, n_pods=1500, identical=True, cond_move=True),
    "one_zero_request": dict(seed=17, n_nodes=40, n_pods=600, half_zero_every=3),
    "one_zero_request_identical": dict(seed=18, n_nodes=300, n_pods=2000, identical=True, half_zero_every=5),
    # round 6: the fitting pods' pruned scans over the fit pass's block bounds, with 64-, 128- and
    # 256-node blocks (the bound reductions span 16, 32 and 64 lanes), ties across blocks
    "pruned_blocks_128": dict(seed=19, n_nodes=5000, n_pods=1500, cycle=5.0, tiny_every=25),
    "pruned_blocks_128_identical": dict(seed=20, n_nodes=4500, n_pods=1500, identical=True, tiny_every=20),
    "pruned_blocks_256": dict(seed=23, n_nodes=9000, n_pods=1500, removals=True, tiny_every=40),
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
    # one shared read per tile of 8 attempts, plus the rescans of a few lane shares
    assert k["nodes_read"] < 0.25 * 64 * k["attempts"], k


def test_tiles_place_without_full_scans():
    """With the best-node tiles (the variant run below), placements inside tiles cost no full read each:
    fewer entries read than one cache per placement (the fit-only tiles read 1.4 caches per placement
    here)."""
    if not os.environ.get("K10S_TILE_BEST_VARIANT"):
        pytest.skip("runs inside test_tile_best_variant_host")
    scn = backlog_scenario(22, n_nodes=700, n_pods=3000)
    od, eng = parity.run_pair(HostEngine, scn, max_time=1e6, log=False)
    assert parity.compare(od, eng, log=False) == []
    k = eng.results()[0]["counters"]
    assert k["nodes_read"] < 700 * k["placements"], k


def test_tile_best_variant_host():
    """The best-node tiles (K10S_TILE_BEST=1, a measured-and-not-kept knob: k10s_engine.h) stay exact:
    the host build with them on for every cycle (K10S_TILE_ALWAYS=1) runs this file's host cases and
    the host fuzz sweep against the oracle in a child process."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hc = os.path.join(repo, "tests", "hostcheck")
    out = os.path.join(repo, "build", f"libk10s_hostcheck_tilebest_{os.getpid()}.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-w", "-DK10S_TILE_BEST=1",
                           "-DK10S_TILE_ALWAYS=1", "-shared", "-o", out, os.path.join(hc, "hostcheck.cpp"),
                           os.path.join(repo, "kubernetriks_amd", "csrc", "k10s_builder.cpp")])
    try:
        env = dict(os.environ, K10S_HOSTCHECK_LIB=out, K10S_TILE_BEST_VARIANT="1")
        r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-n", "4", "-m", "not gpu", "-p", "no:cacheprovider",
                            os.path.join(repo, "tests", "test_cycle_tile.py"), os.path.join(repo, "tests", "test_engine_parity.py"),
                            "-k", "(cycle_tiles_match_oracle or fuzz_host or tiles_replace or place_without) and not variant "
                                  "and not pruned_blocks"],
                           env=env, cwd=repo, capture_output=True, text=True, timeout=1200)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    finally:
        os.unlink(out)


def test_tile_pruned_scans_read_less_host():
    """Round 6: a tile's pods that fit scan the blocks whose bound can still win (tile_scan_pruned,
    the K10S_TILE_PRUNE=1 knob: measured and not kept) instead of the whole cache.  The host build with
    it gives the same results as the default and reads fewer node-cache entries; it also runs this
    file's host cases."""
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hc = os.path.join(repo, "tests", "hostcheck")
    out = os.path.join(repo, "build", f"libk10s_hostcheck_prune_{os.getpid()}.so")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-ffp-contract=off", "-w", "-DK10S_TILE_PRUNE=1",
                           "-shared", "-o", out, os.path.join(hc, "hostcheck.cpp"),
                           os.path.join(repo, "kubernetriks_amd", "csrc", "k10s_builder.cpp")])
    try:
        import ctypes
        import hostcheck_bridge as hb
        scn = backlog_scenario(24, n_nodes=700, n_pods=3000)
        a = HostEngine(scn, 1)
        a.run_until_all_finished(1e6)
        L = ctypes.CDLL(out)
        saved = hb._lib, hb.LIB_PATH
        try:
            hb._lib, hb.LIB_PATH = None, out
            os.environ["K10S_HOSTCHECK_LIB"] = out
            b = HostEngine(scn, 1)
            b.run_until_all_finished(1e6)
            ra, rb = a.results()[0], b.results()[0]
        finally:
            hb._lib, hb.LIB_PATH = saved
            os.environ.pop("K10S_HOSTCHECK_LIB", None)
        del L
        ka, kb = dict(ra["counters"]), dict(rb["counters"])
        na, nb = ka.pop("nodes_read"), kb.pop("nodes_read")
        assert ka == kb and parity.feq(ra["time"], rb["time"])
        assert nb < 0.95 * na, (na, nb)
        import sys
        env = dict(os.environ, K10S_HOSTCHECK_LIB=out)
        r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-n", "4", "-m", "not gpu", "-p", "no:cacheprovider",
                            os.path.join(repo, "tests", "test_cycle_tile.py"), "-k", "cycle_tiles_match_oracle"],
                           env=env, cwd=repo, capture_output=True, text=True, timeout=1200)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    finally:
        os.unlink(out)
