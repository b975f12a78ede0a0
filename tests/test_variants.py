"""Variant builds of the same engine source against the product build (a K10S_PROF build
once hung on the c5_autoscaled slice, so instrumentation is not trusted to be semantics-neutral
until shown).  Each variant library (built in-tree by __graft_entry__.build()) runs the same 64-replica
c5_autoscaled slice in budgeted launches, in its own process with K10S_LIB set, and must end every
replica with the product build's status, error code, clock bits and every counter; the product
build's rows are in turn checked against the oracle for two replicas (one of which hits a reference
panic in that workload).  Variants:
* prof        K10S_PROF=1: cycle attribution (wider header, 106 VGPRs, 4 waves/SIMD, per-lane
              source dispatch in the compiled loop);
* exec_check  K10S_EXEC_CHECK=3: EXEC guards at every lane-parallel helper and bounded sift loops (a
              guard that fires stops the replica with K10S_ERR_EXEC_GUARD: none may);
* full_scan   K10S_FRONT=0: the screened full scan instead of the per-block Pareto fronts, on a C3
              slice (4,096 nodes and no autoscaler, so the product build's fronts are on); every row
              must match except the engine-only node-cache entries read (counter 16)."""
import json
import os
import subprocess
import sys

import pytest

import oracle_jobs
import parity

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SLICE = ["c5_autoscaled", "64", "4096", "16384", "20000"]
SLICE_C3 = ["c3", "64", "4096", "16384", "20000"]
VARIANTS = {"prof": ("build/libk10s_prof.so", SLICE), "exec_check": ("build/libk10s_EXEC_CHECK3.so", SLICE),
            "full_scan": ("build/libk10s_FRONT0.so", SLICE_C3)}
NODES_READ = 16   # K10S_C_NODES_READ: engine-only, differs by scan design


def _run(lib=None, timeout=240, slice_=SLICE):
    env = dict(os.environ)
    if lib:
        env["K10S_LIB"] = lib
    p = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tools", "variant_run.py"), *slice_], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])


_PRODUCT = {}


def _product(slice_):
    key = tuple(slice_)
    if key not in _PRODUCT:
        _PRODUCT[key] = _run(slice_=slice_)
    return _PRODUCT[key]


@pytest.fixture(scope="module")
def product_rows():
    return _product(SLICE)


@pytest.mark.gpu
def test_product_slice_matches_oracle(product_rows):
    import argparse

    import bench
    from kubernetriks_amd import ensemble
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.native import Engine
    from kubernetriks_amd.scenario import scenario_bulk
    a = argparse.Namespace(workload="c5_autoscaled", nodes=4096, pods=16384, arrival_window=1200.0, replicas=64,
                           score_plugins="least")
    cfg, cluster, workload, _, sweep = bench.build_workload(a)
    scn, blob = scenario_bulk(cfg, cluster, workload)
    params = ensemble.shard_params(Engine(scn, 1, pods_blob=blob).default_params(), 64, 0, base_seed=123,
                                   perturb=True, sweep=sweep)
    rows = product_rows["rows"]
    panicked = [r for r in range(64) if rows[r]["status"] == 2]
    check = sorted({0, panicked[0] if panicked else 63})
    ods = oracle_jobs.replay_many([wl.replica_scenario(cfg, cluster, workload, params[r]) for r in check], 1e7)
    for r, od in zip(check, ods):
        assert od["panicked"] == (rows[r]["status"] == 2), r
        assert od["counters"]["events"] == rows[r]["counters"][14], r
        assert od["counters"]["placements"] == rows[r]["counters"][12], r


@pytest.mark.gpu
@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_variant_build_matches_product(variant):
    lib, slice_ = VARIANTS[variant]
    if not os.path.exists(os.path.join(REPO, lib)):
        pytest.fail(f"{lib} not built (__graft_entry__.build() builds it)")
    product_rows = _product(slice_)
    got = _run(lib, slice_=slice_)
    assert got["engine"] != product_rows["engine"]
    # the library is the variant of THESE sources, not a stale one from an earlier build
    from kubernetriks_amd.build import build_id
    import __graft_entry__ as ge
    extra = [x for x, out in ge.VARIANT_BUILDS if lib.endswith(out)][0]
    assert got["engine"].endswith("build " + build_id(extra)), (got["engine"], build_id(extra))
    for r, (a, b) in enumerate(zip(got["rows"], product_rows["rows"])):
        if variant == "full_scan":
            a, b = dict(a), dict(b)
            a["counters"] = a["counters"][:NODES_READ] + a["counters"][NODES_READ + 1:]
            b["counters"] = b["counters"][:NODES_READ] + b["counters"][NODES_READ + 1:]
        assert a == b, (variant, r, a, b)
    assert sum(x["counters"][14] for x in got["rows"]) == sum(x["counters"][14] for x in product_rows["rows"])
