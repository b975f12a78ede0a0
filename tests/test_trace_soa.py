"""Streaming Alibaba CSV -> K10SPOD1 converter (kubernetriks_amd/trace_soa.py).

Pinned against the object path (scenario.alibaba_workload_trace_from_csv + pods_blob, which
restates workload.rs:56-142) byte for byte, and end to end through the host build of the engine.
The CSV rows in REF_* are the data rows of the reference's own parsing tests
(src/trace/alibaba_cluster_trace_v2017/workload.rs:224-226, 247-249, 269-272, 293-295).
"""
import io
import random

import pytest

import parity
from hostcheck_bridge import HostEngine
from kubernetriks_amd import trace_soa
from kubernetriks_amd import workloads as wl
from kubernetriks_amd.scenario import (GenericWorkloadTrace, SimulationConfig, alibaba_workload_trace_from_csv,
                                       pods_blob, scenario_bulk, scenario_text)

REF_INSTANCES = ("41562,41618,120,686,299,Terminated,1,1,1.5,0.29,1.0,1.2\n"
                 "0,,120,686,,Interrupted,1,1,,,,\n"
                 "76058,76058,,,769,Terminated,1,1,0.5,0.5,,\n")
REF_TASKS = ("10718,12897,15,64,2003,Terminated,50,0.01600704061294748\n"
             "6036,6046,4,6,452,Waiting,,\n"
             "1,2,120,686,1,Terminated,100,0.5\n")


def _synthetic_csv(n_inst=3000, n_tasks=200, seed=11, fits=False, no_job_row=False):
    """fits=True keeps every request within a C3 node, so an engine run finishes every pod (a pod that
    can never fit keeps the unschedulable flush cycling until max_time).  no_job_row appends a row
    that passes every filter but has an empty job id (workload.rs:91 unwraps it: an error)."""
    rng = random.Random(seed)
    tasks, inst = [], []
    for t in range(n_tasks):
        cpu = "" if rng.random() < 0.05 else str(rng.choice([50, 100, 200, 400] + ([] if fits else [2 ** 31])))
        mem = "" if rng.random() < 0.05 else repr(rng.choice([0.0, 1e-9, rng.random() * 0.1] + ([] if fits else [3.5e8])))
        tasks.append(f"0,1,{t % 37},{t},5,Terminated,{cpu},{mem}")
    for _ in range(n_inst):
        start = rng.choice([rng.randint(-5, 5000), 100, 100, 0])
        end = start + rng.choice([0, -1, rng.randint(1, 900)])
        task = rng.randint(0, n_tasks + 20)        # some unknown task ids
        cells = [str(start), "" if rng.random() < 0.03 else str(end), str(task % 37),
                 "" if rng.random() < 0.02 else str(task), "9", "Terminated", "1", "1", "", "", "", ""]
        inst.append(",".join(cells))
    if no_job_row:
        tasks.append(f"0,1,3,{n_tasks + 100},5,Terminated,50,0.01")
        inst.append(f"10,20,,{n_tasks + 100},9,Terminated,1,1,,,,")
    return "\n".join(inst) + "\n", "\n".join(tasks) + "\n"


def _object_path_blob(inst_text, task_text):
    w = alibaba_workload_trace_from_csv(inst_text, task_text)
    ev = sorted(w.events, key=lambda e: e.timestamp)     # workload.rs:140, Python's sort is stable
    return pods_blob([(e.timestamp, e.pod) for e in ev]), ev


@pytest.mark.parametrize("data", ["reference_rows", "synthetic", "empty"])
def test_streamed_blob_equals_object_path(data):
    if data == "reference_rows":
        inst, tasks = REF_INSTANCES, REF_TASKS
    elif data == "synthetic":
        inst, tasks = _synthetic_csv()
    else:
        inst, tasks = "", REF_TASKS
    exp, ev = _object_path_blob(inst, tasks)
    got = trace_soa.alibaba_pods_blob(io.StringIO(inst), io.StringIO(tasks))
    assert got == exp
    d = trace_soa.read_pods_blob(got)
    assert d["names"] == [e.pod.name for e in ev]
    assert list(d["ts"]) == sorted(d["ts"])
    assert [int(x) for x in d["cpu"]] == [int(e.pod.cpu) for e in ev]
    assert [int(x) for x in d["ram"]] == [int(e.pod.ram) for e in ev]


def test_reference_rows_values():
    d = trace_soa.read_pods_blob(trace_soa.alibaba_pods_blob(io.StringIO(REF_INSTANCES), io.StringIO(REF_TASKS)))
    # only the first instance survives (workload.rs:63-87); 100 santicores -> 1000 millicores
    assert d["names"] == ["120_686_0"]
    assert list(d["ts"]) == [41562.0] and list(d["duration"]) == [56.0]
    assert int(d["cpu"][0]) == 1000 and int(d["ram"][0]) == 64 * 1024 ** 3


def test_duplicated_task_and_malformed_blob():
    with pytest.raises(ValueError):
        trace_soa.alibaba_pods_blob(io.StringIO(REF_INSTANCES), io.StringIO(REF_TASKS + REF_TASKS))
    # an instance that passes the filters without a job id: both paths refuse it (workload.rs:91)
    inst, tasks = _synthetic_csv(n_inst=50, n_tasks=10, seed=4, no_job_row=True)
    with pytest.raises(ValueError):
        trace_soa.alibaba_pods_blob(io.StringIO(inst), io.StringIO(tasks))
    with pytest.raises(ValueError):
        alibaba_workload_trace_from_csv(inst, tasks)
    blob = trace_soa.alibaba_pods_blob(io.StringIO(REF_INSTANCES), io.StringIO(REF_TASKS))
    for bad in (blob[:-1], b"K10SPODX" + blob[8:], blob[:10], blob + b"x"):
        with pytest.raises(ValueError):
            trace_soa.read_pods_blob(bad)


@pytest.mark.parametrize("bad", ["trailing", "space", "hash", "offset0"])
def test_malformed_blob_rejected_by_engine_and_reader(bad):
    """k10s_engine_create_bulk (host build) and trace_soa.read_pods_blob apply the same rules."""
    from kubernetriks_amd.scenario import Pod
    blob = bytearray(pods_blob([(1.0, Pod("ab", 1, 1, 1.0)), (2.0, Pod("cd", 1, 1, 1.0))]))
    if bad == "trailing":
        blob += b"x"
    elif bad == "space":
        blob[-1:] = b" "
    elif bad == "hash":
        blob[-3:-2] = b"#"
    else:
        p = 16 + 2 * (8 + 4 + 8 + 8)
        blob[p:p + 4] = (1).to_bytes(4, "little")
    blob = bytes(blob)
    with pytest.raises(ValueError):
        trace_soa.read_pods_blob(blob)
    cluster, _ = wl.c3_traces(n_nodes=4, n_pods=1, arrival_window=1.0, seed=5)
    btext, _ = scenario_bulk(SimulationConfig(), cluster, GenericWorkloadTrace([]))
    with pytest.raises(ValueError):
        HostEngine(btext, 1, pods_blob=blob)


def test_file_round_trip(tmp_path):
    inst, tasks = _synthetic_csv(n_inst=500, seed=3)
    (tmp_path / "i.csv").write_text(inst)
    (tmp_path / "t.csv").write_text(tasks)
    blob = trace_soa.alibaba_pods_blob(str(tmp_path / "i.csv"), str(tmp_path / "t.csv"))
    trace_soa.write_pods_blob(str(tmp_path / "p.k10spod"), blob)
    assert trace_soa.load_pods_blob(str(tmp_path / "p.k10spod")) == blob


def _engine(backend):
    if backend == "host":
        return HostEngine
    from kubernetriks_amd.native import Engine
    return Engine


@pytest.mark.parametrize("perturb", [False, True])
@pytest.mark.parametrize("backend", ["host", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_streamed_blob_runs_like_text(backend, perturb):
    """The converter's block fed to k10s_engine_create_bulk: bit-exact with the ORACLE on the same
    pods as scenario text, and identical to the engine's own text run — with pods that can never fit
    a node (2^31 santicores, 3.5e8 x 128 GiB), so the replica retries them until the max_time guard
    (TIME_LIMIT), and with seed-perturbed replicas (the block's sorted position is the perturbation
    key on both paths)."""
    import oracle_jobs
    E = _engine(backend)
    inst, tasks = _synthetic_csv(n_inst=400, n_tasks=60, seed=5)
    blob = trace_soa.alibaba_pods_blob(io.StringIO(inst), io.StringIO(tasks))
    _, ev = _object_path_blob(inst, tasks)
    assert ev
    cfg = SimulationConfig()
    cluster, _ = wl.c3_traces(n_nodes=48, n_pods=1, arrival_window=1.0, seed=5)
    workload = GenericWorkloadTrace(ev)
    text = scenario_text(cfg, cluster, workload)
    btext, _ = scenario_bulk(cfg, cluster, GenericWorkloadTrace([]))
    caps = parity.parity_caps(log=True)
    params = wl.replica_params(E(text, 1).default_params(), 2, base_seed=31, perturb=perturb)
    max_time = 20000.0
    a = E(text, 2, params=params, caps=caps)
    b = E(btext, 2, params=params, caps=caps, pods_blob=blob)
    for e in (a, b):
        e.run_until_all_finished(max_time)
    ods = oracle_jobs.replay_many([wl.replica_scenario(cfg, cluster, workload, p) for p in params], max_time, workers=1)
    for r in range(2):
        assert repr(a.results()[r]) == repr(b.results()[r])
        assert a.placements(r) == b.placements(r)
        assert a.event_log(r) == b.event_log(r)
        assert parity.compare(ods[r], b, r=r, log=False) == [], r
        assert b.results()[r]["status"] == "time_limit"
    unfit = sum(1 for e in ev if e.pod.cpu > 64000 or e.pod.ram > (1 << 37))
    c = b.results()[0]["counters"]
    assert unfit > 0 and c["pods_succeeded"] == len(ev) - unfit and c["attempts"] > c["placements"]


@pytest.mark.parametrize("backend", ["host", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_stall_guard_stops_a_replica_that_cannot_finish(backend):
    """k10s_capacities.stall_guard: once only periodic ticks are pending, a replica whose remaining
    pods can never fit stops with K10S_REPLICA_STALLED instead of cycling to max_time; up to that
    point it is the run without the guard (a prefix of its event log)."""
    E = _engine(backend)
    inst, tasks = _synthetic_csv(n_inst=300, n_tasks=40, seed=8)
    blob = trace_soa.alibaba_pods_blob(io.StringIO(inst), io.StringIO(tasks))
    cfg = SimulationConfig()
    cluster, _ = wl.c3_traces(n_nodes=32, n_pods=1, arrival_window=1.0, seed=8)
    btext, _ = scenario_bulk(cfg, cluster, GenericWorkloadTrace([]))
    caps = parity.parity_caps(log=True)
    full = E(btext, 1, caps=caps, pods_blob=blob)
    full.run_until_all_finished(1e5)
    caps.stall_guard = 1
    g = E(btext, 1, caps=caps, pods_blob=blob)
    g.run_until_all_finished(1e5)
    rf, rg = full.results()[0], g.results()[0]
    assert rf["status"] == "time_limit" and rg["status"] == "stalled"
    assert rg["time"] < rf["time"] and rg["counters"]["events"] < rf["counters"]["events"] / 10
    log_g = g.event_log(0)
    assert full.event_log(0)[:len(log_g)] == log_g
    for k in ("placements", "pods_succeeded", "terminated_pods"):
        assert rg["counters"][k] == rf["counters"][k], k
    # a replica that does finish is not affected by the guard
    c2, w2 = wl.c3_traces(n_nodes=16, n_pods=40, arrival_window=30.0, seed=2)
    scn = scenario_text(cfg, c2, w2)
    h = E(scn, 1, caps=caps)
    h.run_until_all_finished(1e6)
    assert h.results()[0]["status"] == "finished"


@pytest.mark.parametrize("backend", ["host", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_stall_guard_waits_for_the_flush_under_conditional_move(backend):
    """The conditional move (scheduler.rs:210-233) requeues after a pod finish only the waiting pods
    that fit the resources that finish freed.  Pods of 6 and 4 CPU finish one after the other on a
    10-CPU node: the waiting 8-CPU pod fits neither finish's budget, so it waits for the 300-s
    flush (188-203) with only the periodic ticks pending.  The guard must not call that a stall:
    the replica runs to RunUntilAllPodsAreFinished exactly like the oracle.  A pod that fits no
    node at all still stalls it under the same flag."""
    import oracle_bridge as ob
    from kubernetriks_amd.scenario import GenericClusterTrace, Node, Pod
    E = _engine(backend)
    cfg = SimulationConfig(enable_unscheduled_pods_conditional_move=True)
    cluster = GenericClusterTrace().create_node(0.0, Node("node_10cpu", 10000, 64 << 30))
    for extra, want in ((None, "finished"), (Pod("pod_never_fits", 12000, 1 << 30, 30.0), "stalled")):
        w = GenericWorkloadTrace()
        w.create_pod(1.0, Pod("pod_a6", 6000, 8 << 30, 100.0))
        w.create_pod(1.0, Pod("pod_b4", 4000, 8 << 30, 150.0))
        w.create_pod(2.0, Pod("pod_c8", 8000, 8 << 30, 50.0))
        if extra is not None:
            w.create_pod(3.0, extra)
        scn = scenario_text(cfg, cluster, w)
        caps = parity.parity_caps(log=True)
        caps.stall_guard = 1
        eng = E(scn, 1, caps=caps)
        eng.run_until_all_finished(1e5)
        r = eng.results()[0]
        assert r["status"] == want, r["status"]
        assert r["counters"]["requeued"] >= 1 and r["counters"]["flushed"] >= 1
        if want == "finished":
            o = ob.OracleSim(scn, log=True)
            st = o.run_until_all_finished(1e5)
            od = o.result(placements=True, log=True)
            od["status_name"] = parity.ORACLE_STATUS[st]
            assert parity.compare(od, eng) == []
            assert r["counters"]["pods_succeeded"] == 3
        else:
            assert r["counters"]["pods_succeeded"] == 3 and r["time"] < 2000.0


def test_perturb_blob_matches_perturb_pod():
    import math
    from kubernetriks_amd.scenario import Pod
    rng = random.Random(9)
    pods = [(float(rng.randint(0, 99)), Pod(f"p{i}", rng.choice([0, 1, 1000, 2 ** 32 - 1]),
                                            rng.choice([0, 15, 2 ** 64 - 1, rng.getrandbits(40)]),
                                            None if i % 7 == 0 else rng.random() * 1e4)) for i in range(301)]
    blob = pods_blob(pods)
    for seed, off in ((123, 0), (2 ** 64 - 1, 17)):
        d = trace_soa.read_pods_blob(trace_soa.perturb_pods_blob(blob, seed, off))
        for k, (_, p) in enumerate(pods):
            cpu, ram, dur = wl.perturb_pod(seed, off + k, p.cpu, p.ram, p.duration)
            assert (int(d["cpu"][k]), int(d["ram"][k])) == (cpu, ram), k
            got = float(d["duration"][k])
            assert (dur is None and math.isnan(got)) or got == dur, k


# ---- the cluster side: server_event.csv -> K10SNOD1 ------------------------------------------------
REF_MACHINES = ("49380,618,softerror,machine_fail,0,0,0\n"            # cluster.rs:152 (never added: skipped)
                "0,924,add,,64,0.6899697150104833,0.09572460286727773\n")   # cluster.rs:172


def _synthetic_machines(n=300, seed=3):
    rng = random.Random(seed)
    rows = []
    for m in range(n):
        t = rng.choice([0, 0, rng.randint(1, 90000)])
        rows.append(f"{t},{m},add,,{rng.choice([32, 64, 96])},{rng.random()!r},0.1")
        for _ in range(rng.choice([0, 0, 1, 2])):
            rows.append(f"{rng.randint(0, 90000)},{m},{rng.choice(['softerror', 'harderror'])},machine_fail,0,0,0")
    rows.append("12,99999,softerror,,0,0,0")     # a machine that was never added
    rng.shuffle(rows)
    return "\n".join(rows) + "\n"


@pytest.mark.parametrize("data", ["reference_rows", "synthetic", "empty"])
def test_nodes_blob_equals_object_path(data):
    from kubernetriks_amd.scenario import alibaba_cluster_trace_from_csv, nodes_blob
    text = {"reference_rows": REF_MACHINES, "synthetic": _synthetic_machines(), "empty": ""}[data]
    exp = nodes_blob(alibaba_cluster_trace_from_csv(text).events)
    got = trace_soa.alibaba_nodes_blob(io.StringIO(text))
    assert got == exp
    d = trace_soa.read_nodes_blob(got)
    assert list(d["ts"]) == sorted(d["ts"])
    if data == "reference_rows":
        assert d["names"] == ["alibaba_node_924"] and int(d["cpu"][0]) == 64000 and int(d["op"][0]) == 0
    # a pods block after the nodes block: one create_bulk blob, taken apart again
    pods = trace_soa.alibaba_pods_blob(io.StringIO(REF_INSTANCES), io.StringIO(REF_TASKS))
    assert trace_soa.split_blocks(got + pods) == [got, pods]


def test_malformed_nodes_blob():
    good = trace_soa.alibaba_nodes_blob(io.StringIO(_synthetic_machines(20)))
    bad_op = bytearray(good)
    n = int.from_bytes(good[8:16], "little")
    p_op = 16 + 8 * n + 4 * n + 4 * (n & 1) + 8 * n
    bad_op[p_op:p_op + 4] = (7).to_bytes(4, "little")
    for bad in (good[:-1], good + b"x", bytes(bad_op)):
        with pytest.raises(ValueError):
            trace_soa.read_nodes_blob(bad)
        with pytest.raises(ValueError):
            HostEngine("k10s_scenario 1\nend\n", 1, pods_blob=bad)


@pytest.mark.parametrize("backend", ["host", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_cluster_blob_runs_like_text(backend):
    """A cluster trace with node failures (softerror/harderror removals) as a K10SNOD1 block: the
    engine equals its own text run and the oracle, bit for bit."""
    import oracle_jobs
    from kubernetriks_amd.scenario import alibaba_cluster_trace_from_csv
    E = _engine(backend)
    rows = []
    for m in range(40):
        rows.append(f"0,{m},add,,64,0.6899697150104833,0.1")
    for m in range(0, 40, 7):
        rows.append(f"{200 + m},{m},softerror,machine_fail,0,0,0")
    for m in range(3, 40, 11):
        rows.append(f"{700 + m},{m},harderror,,0,0,0")   # some already removed: skipped
    text = "\n".join(rows) + "\n"
    cluster = alibaba_cluster_trace_from_csv(text)
    _, workload = wl.c3_traces(n_nodes=1, n_pods=400, arrival_window=600.0, seed=6)
    cfg = SimulationConfig()
    full = scenario_text(cfg, cluster, workload)
    btext, blob = scenario_bulk(cfg, cluster, workload, cluster_blob=True)
    assert trace_soa.split_blocks(blob)[0] == trace_soa.alibaba_nodes_blob(io.StringIO(text))
    caps = parity.parity_caps(log=True)
    a = E(full, 1, caps=caps)
    b = E(btext, 1, caps=caps, pods_blob=blob)
    for e in (a, b):
        e.run_until_all_finished(1e6)
    assert repr(a.results()[0]) == repr(b.results()[0]) and a.event_log(0) == b.event_log(0)
    od = oracle_jobs.replay(full)
    assert parity.compare(od, b, log=False) == []
    assert b.results()[0]["counters"]["pods_succeeded"] == 400
