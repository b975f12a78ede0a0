"""Oracle runs as picklable jobs for process pools (TEST INFRASTRUCTURE ONLY).

The GPU parity tests at the full 4,096-node C3 shape replay several replicas through the CPU oracle;
each replay takes seconds, so they run in parallel worker processes (spawned: no GPU state is
inherited).  Each job materializes one replica's scenario (its seed-perturbed trace) and returns
the oracle's result dict with placements.
"""
from __future__ import annotations

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def replay(scenario: str, max_time: float = 1e7) -> dict:
    import oracle_bridge as ob
    import parity
    o = ob.OracleSim(scenario)
    st = o.run_until_all_finished(max_time)
    od = o.result(placements=True)
    od["status_name"] = parity.ORACLE_STATUS[st] if not od["panicked"] else "error"
    return od


def _usable_cores() -> int:
    """The cgroup CPU quota when there is one (16 on the GPU box, whose os.cpu_count() shows the whole
    machine), else the affinity set."""
    import math
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(math.ceil(int(q) / int(period)))))
    except (OSError, ValueError):
        pass
    return n


def replay_many(scenarios, max_time: float = 1e7, workers: int = 0):
    """Oracle results for several scenarios, in order, over a spawned process pool."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    n = workers or min(len(scenarios), 16, _usable_cores())
    if n <= 1:
        return [replay(s, max_time) for s in scenarios]
    with ProcessPoolExecutor(max_workers=n, mp_context=mp.get_context("spawn")) as ex:
        return list(ex.map(replay, scenarios, [max_time] * len(scenarios)))
