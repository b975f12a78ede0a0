"""The event loop's screened scan (k10s_engine.h scan_lanes_screen, K10S_SCAN_SCREEN=1, the default
build's scheduling cycle): a single-precision, division-free test drops nodes that provably cannot
be the (score, last index) argmax; every other fitting node is scored exactly.

* CPU: the screen is sound at and around its threshold over the whole u32 cpu / u64 ram range (a
  node it drops scores strictly below the node the threshold came from, with the host score that
  is bit-identical to the device's); a lane-by-lane model of the device algorithm (per-lane exact
  best, per-step wave threshold, same-allocatables shortcut) picks the reference's argmax
  (kube_scheduler.rs:140-148) on the adversarial node sets of test_scan_adversarial.
* GPU: those node sets as 4,096-node clusters under a pod stream, engine vs oracle event for event.
"""
import ctypes
import random

import pytest

import parity
from hostcheck_bridge import HostEngine
from hostcheck_bridge import lib as hclib
from kubernetriks_amd.scenario import GenericClusterTrace, GenericWorkloadTrace, Node, Pod, SimulationConfig, scenario_text
from test_scan_adversarial import EPS, U64, adversarial_problems, la, reference_argmax


def _hc():
    L = hclib()
    L.hc_scan_screen.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float]
    L.hc_scan_screen.restype = ctypes.c_int
    L.hc_screen_u.argtypes = [ctypes.c_double]
    L.hc_screen_u.restype = ctypes.c_float
    return L


def _rand_req(rng, cap_c, cap_r):
    rc = rng.choice([1, rng.randint(1, cap_c), max(1, cap_c // 2), 500, 64000])
    rr = rng.choice([1, rng.randint(1, cap_r), max(1, cap_r // 3), 1 << 30, 123456789])
    return min(rc, cap_c), min(rr, cap_r)


def test_screen_sound_near_threshold():
    """Nodes built to sit within a few eps of the threshold (u(x) - u(y) in [-eps, 3 eps]) and random
    ones: every node the screen drops scores strictly below y; it drops nearly all nodes more than
    2.2 eps above (so it does prune)."""
    L = _hc()
    rng = random.Random(7)
    dropped = far = far_dropped = 0
    for _ in range(1500):
        B = rng.choice([64000, 1000, rng.randint(1, (1 << 32) - 1), (1 << 32) - 1, rng.randint(1, 200)])
        S = rng.choice([rng.randint(1, 1 << 40), rng.randint(1 << 53, U64), U64, 137438953472, rng.randint(1, 5000)])
        rc, rr = _rand_req(rng, B, S)
        sy = la(B, S, rc, rr)
        thr = L.hc_screen_u(sy)
        uy = rc / B + rr / S
        for _ in range(12):
            A = min(rng.choice([rng.randint(rc, max(rc, 2 * B)), B, rc]), (1 << 32) - 1)
            rest = uy + rng.uniform(-1.0, 3.0) * EPS - rc / A
            if rest <= 0:
                continue
            R = int(rr / rest)
            for R2 in (R - 1, R, R + 1, rng.randint(rr, max(rr, 2 * S))):
                if not (rr <= R2 <= U64) or R2 < 1:
                    continue
                if L.hc_scan_screen(A, R2, rc, rr, thr):
                    dropped += 1
                    assert la(A, R2, rc, rr) < sy, (A, R2, rc, rr, B, S)
                if rc / A + rr / R2 > uy + 2.2 * EPS:
                    far += 1
                    far_dropped += L.hc_scan_screen(A, R2, rc, rr, thr)
    assert dropped > 5000
    assert far_dropped >= 0.99 * far


def test_screen_keeps_everything_before_the_first_threshold():
    L = _hc()
    assert not L.hc_scan_screen(64000, 1 << 37, 500, 1 << 30, float("inf"))
    assert not L.hc_scan_screen((1 << 32) - 1, U64, 1, 1, float("inf"))


def screen_model(L, cpu, ram, present, rc, rr, stats=None):
    """The chosen index (or -1): scan_lanes_screen step by step on 64 lanes."""
    N = len(cpu)
    lanes = [{"s": None, "n": -1, "a": 0, "r": 0, "u": float("inf")} for _ in range(64)]
    thr = float("inf")
    scored = 0
    for base in range(0, N, 256):
        for lane, st in enumerate(lanes):
            for j in range(4):
                n = base + 4 * lane + j
                if n >= N or not present[n] or not (rc <= cpu[n] and rr <= ram[n]):
                    continue
                a, r = cpu[n], ram[n]
                if a == st["a"] and r == st["r"]:
                    st["n"] = n
                elif not L.hc_scan_screen(a, r, rc, rr, thr):
                    scored += 1
                    s = la(a, r, rc, rr)
                    if st["s"] is None or s >= st["s"]:
                        st.update(s=s, n=n, a=a, r=r)
                    st["u"] = min(st["u"], L.hc_screen_u(s))
        thr = min(st["u"] for st in lanes)
    if stats is not None:
        stats["scored"] = stats.get("scored", 0) + scored
        stats["nodes"] = stats.get("nodes", 0) + N
    best = [(st["s"], st["n"]) for st in lanes if st["n"] >= 0]
    return max(best)[1] if best else -1


def test_screen_model_matches_reference_argmax():
    L = _hc()
    stats = {}
    for seed in range(3):
        for cpu, ram, present, rc, rr in adversarial_problems(seed, N=2048, count=16):
            if rc == 0 or rr == 0:
                continue
            assert screen_model(L, cpu, ram, present, rc, rr, stats) == reference_argmax(cpu, ram, present, rc, rr)
    assert stats["scored"] < 0.8 * stats["nodes"]


def _cluster_scenario(cpu, ram, n_pods, seed):
    """The node set as a cluster (all nodes at t=0; capacities >= 1) and a pod stream whose requests
    are the set's own (rc, rr)-like small requests, so consecutive attempts see the near-tie sets
    change one reservation at a time."""
    rng = random.Random(seed)
    c = GenericClusterTrace()
    for i, (a, r) in enumerate(zip(cpu, ram)):
        c.create_node(0.0, Node(f"node_{i:05d}", max(int(a), 1), max(int(r), 1)))
    w = GenericWorkloadTrace()
    for i in range(n_pods):
        w.create_pod(float(1 + i // 20), Pod(f"pod_{i:05d}", rng.choice([1, 500, 1000]),
                                             rng.choice([1, 123456789, 1 << 30]), float(rng.randint(50, 400))))
    return scenario_text(SimulationConfig(), c, w)


def _engine(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


@pytest.mark.parametrize("backend", ["host", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_adversarial_clusters_in_the_event_loop(backend):
    kinds = [0, 1, 2, 3, 4, 5]       # ascending ram, identical, near ties, within eps, huge ram, C3-like
    probs = adversarial_problems(17, N=4096 if backend == "gpu" else 512, count=8)
    for k in kinds:
        cpu, ram, _, _, _ = probs[k]
        scn = _cluster_scenario(cpu, ram, 240 if backend == "gpu" else 80, seed=k)
        od, eng = parity.run_pair(_engine(backend), scn, max_time=50000.0)
        assert parity.compare(od, eng) == [], k
