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
        local = [0.0] * NUM_COUNTERS
        for r in eng.raw_results():
            for k in range(NUM_COUNTERS):
                local[k] += float(r.counters[k])
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
    tot = [0.0] * NUM_COUNTERS
    for r in eng.raw_results():
        for k in range(NUM_COUNTERS):
            tot[k] += float(r.counters[k])
    assert got["summed"] == tot
    assert got["max"] == [1.0, 1.5]
    # the merged estimators are a proper pooling of the replicas' samples
    pd = want["timings"]["pod_duration"]
    assert pd["n"] == sum(int(r.est[0].n) for r in eng.raw_results())
    assert not math.isnan(pd["mean"]) and pd["min"] <= pd["mean"] <= pd["max"]
