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


def _synthetic_csv(n_inst=3000, n_tasks=200, seed=11, fits=False):
    """fits=True keeps every request within a C3 node, so an engine run finishes every pod (a pod that
    can never fit keeps the unschedulable flush cycling until max_time)."""
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
    blob = trace_soa.alibaba_pods_blob(io.StringIO(REF_INSTANCES), io.StringIO(REF_TASKS))
    for bad in (blob[:-1], b"K10SPODX" + blob[8:], blob[:10], blob + b"x"):
        with pytest.raises(ValueError):
            trace_soa.read_pods_blob(bad)


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


@pytest.mark.parametrize("backend", ["host", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_streamed_blob_runs_like_text(backend):
    """The converter's block fed to k10s_engine_create_bulk == the same pods as scenario text."""
    E = _engine(backend)
    inst, tasks = _synthetic_csv(n_inst=400, n_tasks=60, seed=5, fits=True)
    blob = trace_soa.alibaba_pods_blob(io.StringIO(inst), io.StringIO(tasks))
    _, ev = _object_path_blob(inst, tasks)
    assert ev
    cfg = SimulationConfig()
    cluster, _ = wl.c3_traces(n_nodes=48, n_pods=1, arrival_window=1.0, seed=5)
    text = scenario_text(cfg, cluster, GenericWorkloadTrace(ev))
    btext, _ = scenario_bulk(cfg, cluster, GenericWorkloadTrace([]))
    caps = parity.parity_caps(log=True)
    a = E(text, 2, caps=caps)
    b = E(btext, 2, caps=caps, pods_blob=blob)
    for e in (a, b):
        e.run_until_all_finished(1e6)
    for r in range(2):
        assert repr(a.results()[r]) == repr(b.results()[r])
        assert a.placements(r) == b.placements(r)
        assert a.event_log(r) == b.event_log(r)
    c = a.results()[0]["counters"]
    assert c["placements"] == len(ev) and c["pods_succeeded"] == len(ev)


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
