"""The N>1 path on CPU: two gloo ranks each run their shard of the job (ensemble.shard_params) on
the host-check engine and combine with ensemble.ensemble_summary / sum_over_ranks / max_over_ranks
— the same calls bench.py makes over RCCL.  The 2-rank summary must equal the 1-rank run of the same
replicas bit for bit (counters, estimator bits, status histogram)."""
import json
import math
import multiprocessing as mp
import os
import socket
import struct
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _canon(x):
    """JSON-safe, bit-exact form of a summary dict (floats as hex, NaN included)."""
    if isinstance(x, float):
        return struct.pack("<d", x).hex()
    if isinstance(x, dict):
        return {k: _canon(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_canon(v) for v in x]
    return x


def _scenario():
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    from kubernetriks_amd import workloads as wl
    from kubernetriks_amd.scenario import SimulationConfig, scenario_text
    c, w = wl.c3_traces(n_nodes=96, n_pods=200, arrival_window=120.0, seed=3)
    return scenario_text(SimulationConfig(), c, w)


def _run_shard(R, rank):
    from hostcheck_bridge import HostEngine
    from kubernetriks_amd import ensemble
    scn = _scenario()
    probe = HostEngine(scn, 1)
    params = ensemble.shard_params(probe.default_params(), R, rank, base_seed=77)
    eng = HostEngine(scn, R, params=params)
    eng.run_until_all_finished(1e6)
    return eng


def _worker(rank, world, port, R, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    import torch.distributed as dist
    from kubernetriks_amd import ensemble
    from kubernetriks_amd.native import NUM_COUNTERS
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = _run_shard(R, rank)
        summary = ensemble.ensemble_summary(eng.raw_results()).as_dict()
        local = [0] * NUM_COUNTERS
        for r in eng.raw_results():
            for k in range(NUM_COUNTERS):
                local[k] += int(r.counters[k])
        summed = ensemble.sum_over_ranks(local)
        mx = ensemble.max_over_ranks([float(rank), 1.5])
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump({"summary": _canon(summary), "summed": summed, "max": mx}, f)
    finally:
        dist.destroy_process_group()


def test_two_gloo_ranks_equal_one_rank(tmp_path):
    R = 3
    out = str(tmp_path / "rank0.json")
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, 2, port, R, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = json.load(open(out))

    # the same 2R replicas in one process (rank 0 of a 1-rank job with 2R replicas per rank)
    sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
    from kubernetriks_amd import ensemble
    from kubernetriks_amd.native import NUM_COUNTERS
    eng = _run_shard(2 * R, 0)
    want = ensemble.ensemble_summary(eng.raw_results()).as_dict()
    assert got["summary"] == _canon(want)
    assert want["replicas"] == 2 * R and want["counters"]["placements"] > 0
    # histograms went through the cross-rank SUM all-reduce and count every estimator sample
    for k, t in want["timings"].items():
        assert sum(want["histograms"][k]) == t["n"] > 0, k
    tot = [0] * NUM_COUNTERS
    for r in eng.raw_results():
        for k in range(NUM_COUNTERS):
            tot[k] += int(r.counters[k])
    assert got["summed"] == tot
    assert got["max"] == [1.0, 1.5]
    # the merged estimators are a proper pooling of the replicas' samples
    pd = want["timings"]["pod_duration"]
    assert pd["n"] == sum(int(r.est[0].n) for r in eng.raw_results())
    assert not math.isnan(pd["mean"]) and pd["min"] <= pd["mean"] <= pd["max"]


def _bench(args, env_extra=None):
    import subprocess
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=600)
    return p


def test_bench_gpus_2_launches_two_ranks():
    """bench.py --gpus 2 (no WORLD_SIZE): the parent spawns 2 rank processes that combine over
    torch.distributed; their int64 counter totals equal one rank running both shards' replicas."""
    common = ["--selftest-host", "--nodes", "64", "--pods", "120", "--arrival-window", "60", "--steps", "1",
              "--warmup", "0", "--no-cpu-baseline"]
    p2 = _bench(["--gpus", "2", "--replicas", "2", *common])
    assert p2.returncode == 0, p2.stderr[-2000:]
    lines = [json.loads(x) for x in p2.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p2.stdout  # rank 0 prints the one line
    two = lines[0]
    assert two["n_gpus"] == 2 and two["config"]["total_replicas"] == 4
    assert "[rank 1]" in p2.stderr and "[rank 0]" in p2.stderr
    p1 = _bench(["--gpus", "1", "--replicas", "4", *common])
    assert p1.returncode == 0, p1.stderr[-2000:]
    one = json.loads([x for x in p1.stdout.splitlines() if x.startswith("{")][0])
    assert one["n_gpus"] == 1
    for k in ("placements", "attempts", "events", "nodes_scanned"):
        assert isinstance(two["totals"][k], int) and two["totals"][k] == one["totals"][k] > 0, k
    assert two["ensemble"]["counters"] == one["ensemble"]["counters"]
    assert two["totals"]["replica_status"] == one["totals"]["replica_status"] == {"1": 4}


def test_bench_gpus_4_c5_sweep_cells_match_one_rank():
    """bench.py --gpus 4 --workload c5 (4 gloo ranks x 2 replicas, the host-check engine): rank g runs
    sweep cells [2g, 2g + 2) of workloads.c5_params (ensemble.shard_params(sweep=True)), so the job's
    per-replica rows in global order equal one rank running cells 0..7, replica by replica."""
    common = ["--selftest-host", "--workload", "c5", "--nodes", "48", "--pods", "90", "--arrival-window", "50",
              "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--replica-rows"]
    p4 = _bench(["--gpus", "4", "--replicas", "2", *common])
    assert p4.returncode == 0, p4.stderr[-2000:]
    four = json.loads([x for x in p4.stdout.splitlines() if x.startswith("{")][0])
    assert four["n_gpus"] == 4 and four["config"]["total_replicas"] == 8
    p1 = _bench(["--gpus", "1", "--replicas", "8", *common])
    assert p1.returncode == 0, p1.stderr[-2000:]
    one = json.loads([x for x in p1.stdout.splitlines() if x.startswith("{")][0])
    assert four["replica_rows"] == one["replica_rows"]
    rows = one["replica_rows"]["counters"]
    assert len(rows) == 8 and len({tuple(r) for r in rows}) > 1   # the cells differ
    assert four["totals"]["events"] == one["totals"]["events"] > 0


def test_bench_world_size_mismatch_fails():
    p = _bench(["--gpus", "2", "--selftest-host", "--replicas", "1", "--nodes", "8", "--pods", "4", "--steps", "1",
                "--warmup", "0", "--no-cpu-baseline"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


def test_launcher_builds_a_stale_library_once(tmp_path):
    """bench.py --gpus 2 brings a stale engine library up to date in the launcher parent (hipcc only,
    no GPU) before it spawns the ranks, so N ranks never compile into the same paths at once."""
    lib = str(tmp_path / "libk10s.so")          # absent = stale
    common = ["--selftest-host", "--nodes", "32", "--pods", "40", "--arrival-window", "30", "--steps", "1",
              "--warmup", "0", "--no-cpu-baseline", "--replicas", "1"]
    p = _bench(["--gpus", "2", *common], {"K10S_BUILD_OUT": lib})
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stderr.count("[build] compiling") == 1, p.stderr[-2000:]
    assert os.path.getsize(lib) > 0
    assert not [f for f in os.listdir(tmp_path) if ".tmp" in f]   # published by rename
    p2 = _bench(["--gpus", "2", *common], {"K10S_BUILD_OUT": lib})   # up to date now: no compile
    assert p2.returncode == 0 and "[build] compiling" not in p2.stderr


def _build_worker(out, q):
    sys.path.insert(0, REPO)
    import contextlib
    import io
    from kubernetriks_amd.build import build
    err = io.StringIO()
    with contextlib.redirect_stderr(err):
        build(out=out)
    q.put(err.getvalue())


def test_concurrent_builds_compile_once(tmp_path):
    """Three processes find the same library stale at once (ranks under torch.distributed.run): the
    file lock lets one compile and the others reuse its result."""
    out = str(tmp_path / "libk10s_race.so")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_build_worker, args=(out, q)) for _ in range(3)]
    for p in procs:
        p.start()
    logs = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs)
    assert sum(s.count("[build] compiling") for s in logs) == 1, logs
    import ctypes
    lib = ctypes.CDLL(out)
    assert lib.k10s_version


_RCCL_ONE_RANK = r"""
import os, sys
sys.path[:0] = [{repo!r}, os.path.join({repo!r}, "tests")]
import numpy as np, torch, torch.distributed as dist
from kubernetriks_amd import ensemble, workloads as wl
from kubernetriks_amd.native import Engine
from kubernetriks_amd.scenario import SimulationConfig, scenario_text
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="{port}")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
assert dist.get_backend() == "nccl"
c, w = wl.c3_traces(n_nodes=64, n_pods=80, arrival_window=40.0, seed=4)
scn = scenario_text(SimulationConfig(), c, w)
params = ensemble.shard_params(Engine(scn, 1).default_params(), 6, 0, base_seed=9)
eng = Engine(scn, 6, params=params)
eng.run_until_all_finished(1e6)
raw = eng.raw_results()
a = ensemble.ensemble_summary(raw).as_dict()
b = ensemble.ensemble_summary(raw, force=True).as_dict()       # all-gather + all-reduce over RCCL
assert repr(a) == repr(b), (a, b)
big = [2 ** 62 + 12345, 3, 0, 2 ** 53 + 1]
assert ensemble.sum_over_ranks(big, force=True) == big           # int64 exact through RCCL
assert ensemble.max_over_ranks([1.5, -2.0], force=True) == [1.5, -2.0]
g = ensemble._gather(np.arange(12, dtype=np.int64).reshape(3, 4))
assert g.tolist() == np.arange(12).reshape(3, 4).tolist()
h = ensemble._all_reduce_sum(np.full((3, 32), 2 ** 40 + 7, dtype=np.int64))
assert (h == 2 ** 40 + 7).all()
dist.destroy_process_group()
print("RCCL_ONE_RANK_OK", a["counters"]["placements"])
"""


@pytest.mark.gpu
def test_rccl_collectives_one_rank_gpu():
    """The nccl (= RCCL over xGMI) branches of ensemble._gather / _all_reduce_sum / sum_over_ranks /
    max_over_ranks / ensemble_summary, forced on a one-rank group on the real GPU: they must give
    exactly the local values (device tensors, int64 counters above 2^53)."""
    import subprocess
    code = _RCCL_ONE_RANK.format(repo=REPO, port=_free_port())
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and "RCCL_ONE_RANK_OK" in p.stdout, (p.stdout[-1000:], p.stderr[-3000:])
