"""Replica sharding over ranks and the end-of-run cross-rank reduction.

Replicas are independent simulations, so a job of W ranks x R replicas gives rank g the replicas
[g*R, (g+1)*R) (seeds base_seed + g*R + i; weak scaling: R per rank).  Nothing is exchanged while
the replicas run.  At the end the ranks combine, over torch.distributed (RCCL over xGMI when the
group is "nccl", gloo on CPU):
  * the per-replica counter rows and estimator rows, all-gathered in rank order (R rows per rank),
    so that metrics.EnsembleSummary merges them in global replica order — the summary of the job
    is bit-identical for any world size;
  * the log2 histograms of pod duration / scheduling latency / queue time (K10S_HIST_BINS bins per
    estimator), summed over the rank's replicas and then all-reduced (SUM) — the RCCL all-reduce of
    metric histograms;
  * scalar timings, max-reduced (`max_over_ranks`).
The reference is single-process (no collective exists there); this is the ensemble layer around it.
"""
from __future__ import annotations

from typing import Optional, Sequence

from . import workloads as wl
from .metrics import EnsembleSummary, estimator_rows
from .native import COUNTER_NAMES, EST_NAMES, HIST_BINS, NUM_COUNTERS, STATUS


def replica_offset(rank: int, replicas_per_rank: int) -> int:
    return rank * replicas_per_rank


def shard_params(defaults, replicas_per_rank: int, rank: int, base_seed: int = 123, perturb: bool = True,
                 sweep: bool = False):
    """k10s_replica_params of rank `rank`'s block: seed-perturbed copies of the scenario (C2/C3), or
    the scheduler/autoscaler parameter sweep (C5) when `sweep`."""
    off = replica_offset(rank, replicas_per_rank)
    if sweep:
        return wl.c5_params(defaults, replicas_per_rank, base_seed=base_seed, replica_offset=off)
    return wl.replica_params(defaults, replicas_per_rank, base_seed=base_seed, perturb=perturb, replica_offset=off)


def _rows(raw_results):
    import numpy as np
    cnt = np.array([[int(r.counters[k]) for k in range(NUM_COUNTERS)] for r in raw_results], dtype=np.int64)
    est = np.array([estimator_rows(r) for r in raw_results], dtype=np.float64).reshape(len(raw_results), len(EST_NAMES), 5)
    st = np.array([int(r.status) for r in raw_results], dtype=np.int64)
    return cnt, est, st


def _dist_group_size(group=None) -> int:
    try:
        import torch.distributed as dist
    except ImportError:
        return 1
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def _gather(arr, group=None):
    """All-gather equal-shaped numpy arrays across the group, concatenated in rank order."""
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(arr)).to(dev)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return torch.cat(parts).cpu().numpy()


def _collective(group, force: bool) -> bool:
    """Run the cross-rank collective: always with more than one rank; with one rank only when
    `force`d and a process group is initialised (so the RCCL path is exercised on one GPU)."""
    n = _dist_group_size(group)
    if n > 1:
        return True
    if not force:
        return False
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def ensemble_summary(raw_results: Sequence, group=None, force: bool = False) -> EnsembleSummary:
    """Summary of every replica of the job (all ranks when torch.distributed is initialised; every
    rank must pass the same number of replicas).  Identical on every rank."""
    cnt, est, st = _rows(raw_results)
    hist = histogram_sum(raw_results)
    if _collective(group, force):
        cnt, est, st = _gather(cnt, group), _gather(est, group), _gather(st, group)
        hist = _all_reduce_sum(hist, group)
    s = EnsembleSummary(COUNTER_NAMES, EST_NAMES)
    for i in range(cnt.shape[0]):
        s.add_replica(cnt[i].tolist(), est[i].tolist(), STATUS.get(int(st[i]), str(int(st[i]))))
    s.set_histograms(hist)
    return s


def gather_rows(raw_results: Sequence, group=None):
    """(counters int64 [R_job, NUM_COUNTERS], estimators f64 [R_job, len(EST_NAMES), 5], status int64 [R_job])
    of every replica of the job in global replica order (all ranks when torch.distributed is
    initialised): per-replica fingerprints, e.g. to check that rank g ran sweep cells [g·R, (g+1)·R)."""
    cnt, est, st = _rows(raw_results)
    if _collective(group, False):
        cnt, est, st = _gather(cnt, group), _gather(est, group), _gather(st, group)
    return cnt, est, st


def histogram_sum(raw_results):
    """(len(EST_NAMES), HIST_BINS) int64: the replicas' estimator histograms summed."""
    import numpy as np
    h = np.zeros((len(EST_NAMES), HIST_BINS), dtype=np.int64)
    for r in raw_results:
        h += np.array([list(r.est[i].hist) for i in range(len(EST_NAMES))], dtype=np.int64)
    return h


def _all_reduce_sum(arr, group=None):
    """Element-wise SUM of an int64 array over the group (RCCL over xGMI for "nccl", gloo on CPU)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.from_numpy(arr.copy()).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.cpu().numpy()


def max_over_ranks(values: Sequence[float], group=None, device: Optional[str] = None, force: bool = False):
    """Element-wise max of a few scalars over the group (the bench's timing reduction)."""
    if not _collective(group, force):
        return list(values)
    import torch
    import torch.distributed as dist
    dev = device or ("cuda" if dist.get_backend(group) == "nccl" else "cpu")
    t = torch.tensor(list(values), dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.cpu().tolist()


def sum_over_ranks(values: Sequence[int], group=None, device: Optional[str] = None, force: bool = False):
    """Element-wise sum of a u64 counter vector over the group (RCCL all-reduce on GPUs), in int64:
    exact for every count below 2^63 (a float64 sum would round above 2^53)."""
    vals = [int(v) for v in values]
    if not _collective(group, force):
        return vals
    import torch
    import torch.distributed as dist
    dev = device or ("cuda" if dist.get_backend(group) == "nccl" else "cpu")
    t = torch.tensor(vals, dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return [int(v) for v in t.cpu().tolist()]
