"""The event loop compiles to uniform control flow in every build variant.

Round 3's K10S_PROF build hung on c5_autoscaled: with the stale-finish skip's heap_pop + sl_refresh
inlined into the source selection loop, the compiler threaded sl_update's lane-0 store into the
loop's back edge and structurized the event loop and the selection loop as divergent loops (EXEC
masked at their back edges), so the wave-parallel helpers could run under a partial EXEC; replica 53
never left its first stale skip.  The skip is now an out-of-line call
(drop_stale_head).  This test compiles each variant's device code (hipcc cross-compiles here, no
GPU) and checks that the only divergent loops of the run kernel are innermost loops that call
nothing: the lane-strided copies and scans (tools/divergent_loops.py).  Since round 5 (VERDICT r04
#3) the same walk covers every device function the run kernel reaches through calls — the handlers,
both scheduling cycles, the move-all requeue, the CA decision, the stale-finish skip: a divergent loop
there may not contain a call or a cross-lane instruction.  The GPU side of the same claim is
tests/test_variants.py."""
import os
import shutil
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import divergent_loops  # noqa: E402

VARIANTS = {
    "product": [],
    "prof": ["-DK10S_PROF=1"],
    "exec_check": ["-DK10S_EXEC_CHECK=3"],
    "prof_beacon": ["-DK10S_PROF=1", "-DK10S_BEACON=1"],
    "split1": ["-DK10S_SPLIT=1"],
}
CASES = [(v, p) for v in VARIANTS for p in (False, True)]


@pytest.fixture(scope="module")
def loops():
    if not shutil.which("hipcc") and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    with ThreadPoolExecutor(max_workers=min(len(CASES), max(1, (os.cpu_count() or 2) // 2))) as ex:
        futs = {c: ex.submit(divergent_loops.compile_and_check, VARIANTS[c[0]], c[1]) for c in CASES}
        return {c: f.result() for c, f in futs.items()}


# out-of-line device functions of the product build that the walk must reach
CALLEES = ["run_scheduling_cycle_t", "run_scheduling_cycle_tiles", "on_api_server", "on_ps", "on_node",
           "s_move_all_dev", "ca_decide", "drop_stale_head", "heap_pop", "on_hpa", "on_ca", "on_metrics"]


@pytest.mark.parametrize("variant,plugins", CASES, ids=[f"{v}{'-plugins' if p else ''}" for v, p in CASES])
def test_event_loop_is_uniform(loops, variant, plugins):
    funcs, got = loops[(variant, plugins)]
    bad = [x for x in got if not x["ok"]]
    assert not bad, bad
    assert got, "expected the header-copy loops (analysis found no loop at all)"
    if variant == "product":
        for name in CALLEES:
            if plugins and name == "run_scheduling_cycle_tiles":
                continue   # the tiled cycle is a packed-cache path: not compiled into the wide copy
            assert any(name in f for f in funcs), (name, funcs)


def test_detects_a_divergent_event_loop():
    """The analysis flags round 3's shape: a structurized loop nested in the event loop."""
    asm = """_Z15k10s_run_kerneljiddmPj:
.LBB1_1:                                ; =>This Inner Loop Header: Depth=1
\tv_add_u32 v0, 1, v0
\ts_andn2_b64 exec, exec, s[4:5]
\ts_cbranch_execnz .LBB1_1
.LBB1_2:                                ; =>This Loop Header: Depth=1
\ts_swappc_b64 s[30:31], s[0:1]
.LBB1_3:                                ;   in Loop: Header=BB1_2 Depth=1
\ts_andn2_b64 exec, exec, s[44:45]
\ts_cbranch_execz .LBB1_4
.LBB1_4:
\ts_branch .LBB1_2
.Lfunc_end1:""".split("\n")
    got = divergent_loops.divergent_loops(asm)
    assert [x["ok"] for x in got] == [True, False]


def test_detects_a_divergent_callee_loop():
    """A callee reached from the kernel with round 3's shape — a divergent loop around a call and a
    DPP reduction — is flagged; an innermost copy loop beside it passes, and so does a divergent
    loop around a nested plain loop (no call, nothing cross-lane)."""
    asm = """_Z15k10s_run_kerneljiddmPj:
\ts_getpc_b64 s[4:5]
\ts_add_u32 s4, s4, _ZN4k10s6calleeERNS_3CtxE@rel32@lo+4
\ts_swappc_b64 s[30:31], s[4:5]
.Lfunc_end1:
_ZN4k10s6calleeERNS_3CtxE:
.LBB2_1:                                ; =>This Inner Loop Header: Depth=1
\tglobal_store_dword v[0:1], v2, off
\ts_andn2_b64 exec, exec, s[4:5]
\ts_cbranch_execnz .LBB2_1
.LBB2_2:                                ; =>This Loop Header: Depth=1
\tv_add_f32_dpp v1, v1, v1 row_shr:1 row_mask:0xf bank_mask:0xf
\ts_getpc_b64 s[6:7]
\ts_add_u32 s6, s6, _ZN4k10s8heap_popERNS_3CtxE@rel32@lo+4
\ts_swappc_b64 s[30:31], s[6:7]
.LBB2_3:                                ;   in Loop: Header=BB2_2 Depth=1
\ts_andn2_b64 exec, exec, s[44:45]
\ts_cbranch_execz .LBB2_4
.LBB2_4:                                ;   in Loop: Header=BB2_2 Depth=1
\ts_branch .LBB2_2
.LBB2_5:                                ; =>This Loop Header: Depth=1
\tv_add_u32 v0, 1, v0
.LBB2_6:                                ;   Parent Loop BB2_5 Depth=1
                                        ; =>  This Inner Loop Header: Depth=2
\tglobal_load_dword v3, v[0:1], off
\ts_cbranch_scc1 .LBB2_6
.LBB2_7:                                ;   in Loop: Header=BB2_5 Depth=1
\ts_andn2_b64 exec, exec, s[8:9]
\ts_cbranch_execnz .LBB2_5
.Lfunc_end2:
_ZN4k10s8heap_popERNS_3CtxE:
\ts_setpc_b64 s[30:31]
.Lfunc_end3:""".split("\n")
    funcs, got = divergent_loops.reachable_divergent_loops(asm)
    assert funcs == ["_Z15k10s_run_kerneljiddmPj", "_ZN4k10s6calleeERNS_3CtxE", "_ZN4k10s8heap_popERNS_3CtxE"]
    assert [(x["header"], x["ok"]) for x in got] == [(".LBB2_1", True), (".LBB2_2", False), (".LBB2_5", True)]
    bad = got[1]
    assert bad["swappc"] == 1 and bad["wave_ops"] == 1
