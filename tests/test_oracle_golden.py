"""Pin the CPU oracle against the golden values held by the reference's own tests
(tests/golden/reference_goldens.json).  Runs on CPU only."""
import json
import math
import os
import struct

import pytest

import oracle_bridge as ob
import scenarios as sc

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.json")))


def f64hex(x: float) -> str:
    return "0x%016x" % struct.unpack("<Q", struct.pack("<d", x))[0]


# ---- scheduler.rs:522-602 ---------------------------------------------------------------
def test_schedule_one_errors():
    s = G["scheduler_unit"]
    for case in ("no_nodes", "zero_request", "no_sufficient"):
        c = s[case]
        st, _ = ob.schedule_one([tuple(n) for n in c["nodes"]], *c["pod"])
        assert st == c["status"], case


def test_schedule_one_correct_node_and_scores():
    c = G["scheduler_unit"]["correct"]
    st, name = ob.schedule_one([tuple(n) for n in c["nodes"]], *c["pod"])
    assert (st, name) == (0, c["node"])
    for n, cpu, ram in c["nodes"]:
        score = ob.least_allocated(cpu, ram, *c["pod"])
        assert f64hex(score) == c["scores_hex"][n]
        assert abs(score - c["scores_approx"][n]) < 0.01


def test_several_pod_scheduling_sequential_packing():
    c = G["scheduler_unit"]["several"]
    name, cpu, ram = c["node"]
    for pcpu, pram, expect in c["pods"]:
        st, chosen = ob.schedule_one([(name, cpu, ram)], pcpu, pram)
        assert st == expect
        if st == 0:
            assert chosen == name
            cpu -= pcpu
            ram -= pram


def test_tie_break_is_last_max_in_name_order_and_nan_first_rule():
    # equal scores: the reference keeps the LAST node in byte order (kube_scheduler.rs:140-148)
    nodes = [("default_node_10", 1000, 1000), ("default_node_2", 1000, 1000), ("a", 1000, 1000)]
    st, name = ob.schedule_one(nodes, 10, 10)
    assert (st, name) == (0, "default_node_2")
    # first filtered node has NaN score (alloc cpu == req cpu == 0) -> it wins regardless
    nodes = [("n0", 0, 1000), ("n1", 100, 5000)]
    st, name = ob.schedule_one(nodes, 0, 10)
    assert (st, name) == (0, "n0")
    # a NaN score elsewhere is never selected
    nodes = [("n0", 100, 5000), ("n1", 0, 1000)]
    st, name = ob.schedule_one(nodes, 0, 10)
    assert (st, name) == (0, "n0")


# ---- queue.rs:86-164 -------------------------------------------------------------------
def test_active_queue_pop_order():
    q = G["queue_order"]
    order = ob.heap_pop_order(q["heap_push_ts"])
    assert [q["heap_push_ts"][i] for i in order] == q["heap_pop_ts"]


def test_unschedulable_key_order():
    q = G["queue_order"]
    entries = [tuple(e) for e in q["unsched_entries"]]
    order = ob.unsched_order(entries)
    assert [entries[i][0] for i in order] == q["unsched_order_names"]


# ---- pod_group.rs / constant.rs ---------------------------------------------------------
def test_pod_group_usage_models():
    u = G["pod_group_usage"]
    for key in ("doc_test", "one_unit"):
        c = u[key]
        r, vals = ob.pod_group_usage(c["model"], c["creation"], [tuple(p) for p in c["polls"]])
        assert r == 0 and vals == c["expect"], key
    c = u["past_panics"]
    r, _ = ob.pod_group_usage(c["model"], c["creation"], [tuple(p) for p in c["polls"]])
    assert r == 1
    c = u["complex"]
    for shift in c["shifts"]:
        polls = [(t + shift, n) for t, n in c["polls"]]
        r, vals = ob.pod_group_usage(c["model"], shift, polls)
        assert r == 0 and vals == c["expect"], shift
    c = u["constant"]
    r, vals = ob.pod_group_usage(c["model"], 0.0, [tuple(p) for p in c["polls"]])
    assert r == 0 and vals == c["expect"]


# ---- simulator.rs:415-533 -----------------------------------------------------------------
def test_max_nodes_in_trace():
    for kinds, expect in G["max_nodes_in_trace"]["cases"]:
        assert ob.max_nodes_in_trace(kinds) == expect


# ---- tests/test_hpa.rs ------------------------------------------------------------------
def test_hpa_pod_group_sizes():
    s = ob.OracleSim(sc.sc_hpa())
    for t, size in G["hpa"]["checkpoints"]:
        s.step_until_time(t)
        r = s.result()
        assert not r["panicked"], r["panic"]
        assert r["hpa_groups"]["pod_group_1"][0] == size, t


# ---- tests/test_pods.rs -----------------------------------------------------------------
def _run(scn):
    s = ob.OracleSim(scn)
    st = s.run_until_all_finished(1e6)
    assert st == 0
    return s.result(placements=True)


def test_pod_arrived_before_a_node():
    r = _run(sc.sc_pod_arrived_before_node())
    rec = r["pods"]["pod_16"]
    assert rec[5] == 1 and rec[2] > 30.0 and not math.isnan(rec[3])


def test_many_pods_running_one_at_a_time():
    r = _run(sc.sc_many_pods_one_at_a_time())
    for i in range(4):
        assert r["pods"][f"pod_{i}"][5] == 1


def test_node_fits_all_pods_run_in_parallel():
    r = _run(sc.sc_node_fits_all_pods())
    fin = [r["pods"][f"pod_{i}"][3] for i in range(3)]
    assert all(r["pods"][f"pod_{i}"][5] == 1 for i in range(3))
    assert fin[0] > fin[1] > fin[2]


@pytest.mark.parametrize("name", ["pod_removals", "pod_removal_concurrent_with_node_removal",
                                  "pod_removed_after_finished"])
def test_pod_counters(name):
    r = _run(sc.ALL_TEST_SCENARIOS[name]())
    for k, v in G["pods"][name].items():
        assert r["counters"][k] == v, k


def test_removed_pod_frees_place_for_other_pod():
    g = G["pods"]["removed_pod_frees_place"]
    s = ob.OracleSim(sc.sc_removed_pod_frees_place())
    s.step_for_duration(100.0)
    assert s.result()["unschedulable_len"] == g["unschedulable_len_at_100"]
    s.step_for_duration(240.0)
    c = s.result()["counters"]
    for k, v in g["after_340"].items():
        assert c[k] == v, k


def test_node_remove_while_pods_were_running():
    g = G["pods"]["node_remove_while_running"]
    s = ob.OracleSim(sc.sc_node_remove_while_running())
    s.step_for_duration(1000.0)
    c = s.result()["counters"]
    for k, v in g["at_1000"].items():
        assert c[k] == v
    s.step_for_duration(2000.0)
    assert s.result()["counters"]["pods_succeeded"] == g["at_3000"]["pods_succeeded"]


def test_node_removed_at_the_same_time_as_assignment():
    g = G["pods"]["node_removed_same_time_as_assignment"]
    s = ob.OracleSim(sc.sc_node_removed_same_time_as_assignment())
    s.step_for_duration(1000.0)
    c = s.result()["counters"]
    for k, v in g["at_1000"].items():
        assert c[k] == v


# ---- tests/test_node_creation.rs, tests/test_default_cluster.rs ----------------------------
def test_node_creation_from_trace_and_default_cluster():
    g = G["node_creation"]
    s = ob.OracleSim(sc.sc_node_creation())
    assert s.result()["node_counts"] == [g["at_init"]] * 3
    s.step_for_duration(1000.0)
    r = s.result(placements=True)
    assert r["node_counts"] == [g["at_1000"]] * 3
    for comp in ("as", "ps", "s"):
        assert [n[0] for n in r["nodes"][comp]] == g["names_at_1000"]


def _nodes(scn):
    s = ob.OracleSim(scn)
    r = s.result(placements=True)
    for comp in ("as", "ps", "s"):
        assert r["nodes"][comp] == r["nodes"]["s"]
    return {n[0]: (n[1], n[2], n[3], n[4]) for n in r["nodes"]["s"]}


def test_default_cluster_without_name_prefix():
    g = G["default_cluster"]["no_prefix"]
    nodes = _nodes(sc.sc_default_cluster_no_prefix())
    assert len(nodes) == g["count"]
    for prefix, lo, hi, cpu, ram in g["groups"]:
        for i in range(lo, hi):
            assert nodes[f"{prefix}{i}"] == (cpu, ram, cpu, ram)


@pytest.mark.parametrize("case,fn", [("no_count", sc.sc_default_cluster_no_count), ("prefix", sc.sc_default_cluster_prefix)])
def test_default_cluster_named(case, fn):
    g = G["default_cluster"][case]
    nodes = _nodes(fn())
    assert len(nodes) == len(g["nodes"])
    for name, cpu, ram in g["nodes"]:
        assert nodes[name] == (cpu, ram, cpu, ram)


# ---- tests/test_determinism.rs: repeated runs are identical -----------------------------------
def test_determinism_repeated_runs_identical():
    scn = sc.sc_c1_generic_example()
    ref = _run(scn)
    for _ in range(3):
        assert _run(scn) == ref
