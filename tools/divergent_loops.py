#!/usr/bin/env python3
"""Divergent loops of the event-loop kernel (tooling; tests/test_uniform_loop.py runs it per build
variant).  Compiles kubernetriks_amd/csrc/k10s_kernels.hip to gfx950 assembly with the given extra
hipcc flags (e.g. -DK10S_PROF=1) and lists, in the run kernel, every loop the compiler structurized
as divergent (its back edge masks EXEC: `s_andn2_b64 exec, exec, ...`) together with whether the
loop body calls a function.  The event loop and the source selection loop must be uniform (scalar
branches only): a divergent structurization there runs the wave-parallel helpers (heap_pop,
sl_update) under a partial EXEC, which is how the K10S_PROF build of round 3 hung.
Only innermost loops that call nothing may be divergent: the lane-strided copies and scans (header
copies before and after the event loop, window refills, node scans).  Prints one JSON object.

Since round 5 every device function the run kernel reaches through calls (the handlers, the
scheduling cycles, s_move_all_dev, ca_decide, drop_stale_head, heap_pop, ...) is walked the same way:
a divergent loop there must also be innermost and call-free, and must not contain a wave-parallel
instruction (DPP, permlane, ds_swizzle/bpermute, mbcnt): under a partial EXEC those read the disabled
lanes' stale values.

Usage: tools/divergent_loops.py [--plugins] [hipcc flags...]"""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "_Z15k10s_run_kerneljiddmPj"


# cross-lane instructions of the wave-parallel helpers (reductions, ballot positions, permutes)
WAVE_OP = re.compile(r"\b(row_\w+|quad_perm|row_bcast\w*|wave_\w+)\b|\bv_permlane|\bds_swizzle|\bds_bpermute|"
                     r"\bds_permute|\bv_mbcnt")


def functions(asm_lines):
    """{symbol: (first line, .Lfunc_end line)} of every function in the assembly."""
    out = {}
    for i, l in enumerate(asm_lines):
        m = re.match(r"^([_A-Za-z][_A-Za-z0-9]*):", l)
        if m and not m.group(1).startswith(".L"):
            for j in range(i + 1, len(asm_lines)):
                if asm_lines[j].startswith(".Lfunc_end"):
                    out[m.group(1)] = (i, j)
                    break
                if re.match(r"^[_A-Za-z][_A-Za-z0-9]*:", asm_lines[j]):
                    break
    return out


def reachable(asm_lines, kernel=KERNEL):
    """The kernel and every function it reaches through calls (s_getpc + @rel32 relocations)."""
    funcs = functions(asm_lines)
    seen, todo = [], [kernel]
    while todo:
        f = todo.pop()
        if f in seen or f not in funcs:
            continue
        seen.append(f)
        st, en = funcs[f]
        for l in asm_lines[st:en]:
            for m in re.finditer(r"([_A-Za-z][_A-Za-z0-9]*)@rel32@lo", l):
                if m.group(1) in funcs and m.group(1) not in seen:
                    todo.append(m.group(1))
    return seen


def divergent_loops(asm_lines, kernel=KERNEL, wave_ops=False):
    st = next(i for i, l in enumerate(asm_lines) if l.startswith(kernel + ":"))
    en = next(i for i in range(st, len(asm_lines)) if asm_lines[i].startswith(".Lfunc_end"))
    labels = {}
    for i in range(st, en):
        m = re.match(r"^(\.LBB\d+_\d+):", asm_lines[i])
        if m:
            labels[m.group(1)] = i
    out = []
    for i in range(st, en):
        if "s_andn2_b64 exec, exec" not in asm_lines[i]:
            continue
        # the back edge: the next branch after the EXEC update jumps to the loop header
        hdr = None
        for j in range(i + 1, min(en, i + 6)):
            m = re.search(r"s_cbranch_execnz (\.LBB\d+_\d+)|s_branch (\.LBB\d+_\d+)", asm_lines[j])
            if m:
                hdr = m.group(1) or m.group(2)
                break
        if hdr is None or hdr not in labels or labels[hdr] > i:
            # structurized form: the header is named in the block comment ("in Loop: Header=BBx_y")
            j = i
            while j > st and not asm_lines[j].startswith(".LBB"):
                j -= 1
            m = re.search(r"Header=BB(\d+_\d+)", asm_lines[j])
            hdr = ".LBB" + m.group(1) if m else None
            if hdr is None and "Loop Header" in asm_lines[j]:
                hdr = asm_lines[j].split(":")[0]
        h = labels.get(hdr, i)
        # the header's loop comment (one line per nesting level) and the loop's blocks: the header
        # block and every block whose comment reads "in Loop: Header=<hdr>"
        comment = []
        j = h
        while j < en and (j == h or asm_lines[j].lstrip().startswith(";")):
            comment.append(asm_lines[j].split(";", 1)[-1].strip())
            j += 1
        body, inside = [], False
        tag = "Header=" + (hdr or "")[2:]
        for j in range(st, en):
            l = asm_lines[j]
            if l.startswith(".LBB") or l.startswith("; %bb."):
                inside = j == h or re.search(re.escape(tag) + r"\b", l) is not None   # BBx_1 is not BBx_15
            if inside:
                body.append(l)
        # with the blocks of every loop nested in it (their comments name only the innermost header)
        nested = loop_tree(asm_lines, st, en)
        full, inside = [], False
        for j in range(st, en):
            l = asm_lines[j]
            if l.startswith(".LBB") or l.startswith("; %bb."):
                b = innermost_header(asm_lines, j, en)
                inside = b is not None and (b == (hdr or "")[2:] or (hdr or "")[2:] in ancestors(nested, b))
            if inside:
                full.append(l)
        inner = any("Inner Loop Header" in x for x in comment)
        swappc = sum("s_swappc_b64" in l for l in full)
        wops = sum(1 for l in full if not l.lstrip().startswith(";") and WAVE_OP.search(l.split(";")[0]))
        # allowed: an innermost loop that calls nothing (lane-strided copies and scans) and, in the
        # callees, runs no cross-lane instruction
        # (the kernel keeps round 4's stricter rule: innermost only; in a callee a divergent loop
        # around a nested loop is fine while nothing in it is cross-lane or a call — e.g. the
        # unschedulable map's insertion shift, whose values the compiler cannot prove uniform)
        out.append({"function": kernel, "line": i - st, "header": hdr, "comment": " | ".join(comment),
                    "blocks_lines": len(full), "swappc": swappc, "wave_ops": wops,
                    "ok": (inner or wave_ops) and swappc == 0 and (not wave_ops or wops == 0)})
    return out


def innermost_header(asm_lines, j, en):
    """'BBx_y' of the innermost loop containing the block that starts at line j (None: no loop)."""
    k = j
    while k < en and (k == j or asm_lines[k].lstrip().startswith(";")):
        c = asm_lines[k].split(";", 1)[-1] if ";" in asm_lines[k] else ""
        if "Loop Header" in c and asm_lines[j].startswith(".LBB"):
            return asm_lines[j].split(":")[0][2:]
        m = re.search(r"in Loop: Header=(BB\d+_\d+)", c)
        if m:
            return m.group(1)
        k += 1
    return None


def loop_tree(asm_lines, st, en):
    """{header 'BBx_y': parent header or None} of the function's loops (from the header comments)."""
    par = {}
    for j in range(st, en):
        l = asm_lines[j]
        if not l.startswith(".LBB"):
            continue
        k, parents, is_hdr = j, [], False
        while k < en and (k == j or asm_lines[k].lstrip().startswith(";")):
            c = asm_lines[k].split(";", 1)[-1] if ";" in asm_lines[k] else ""
            m = re.search(r"Parent Loop (BB\d+_\d+)", c)
            if m:
                parents.append(m.group(1))
            if "Loop Header" in c:
                is_hdr = True
            k += 1
        if is_hdr:
            par[l.split(":")[0][2:]] = parents[-1] if parents else None
    return par


def ancestors(tree, h):
    out = []
    while h in tree and tree[h] is not None:
        h = tree[h]
        out.append(h)
    return out


def reachable_divergent_loops(asm_lines, kernel=KERNEL):
    """divergent_loops over the kernel (calls and nesting checked) and every function it reaches
    (calls, nesting and cross-lane instructions checked).  Returns (functions walked, loops)."""
    fs = reachable(asm_lines, kernel)
    loops = []
    for f in fs:
        loops += divergent_loops(asm_lines, f, wave_ops=(f != kernel))
    return fs, loops


def compile_and_check(flags, plugins=False):
    """Divergent loops of the run kernel of one translation unit (k10s_kernels.hip, or with
    plugins=True the plugin-scoring k10s_kernels_plugins.hip) built with the product flags + flags."""
    src, kernel = ("k10s_kernels_plugins.hip", "_Z23k10s_run_kernel_pluginsjiddmPj") if plugins else \
        ("k10s_kernels.hip", KERNEL)
    out_s = "/tmp/k10s_divergent_loops_%d_%d.s" % (os.getpid(), abs(hash((tuple(flags), plugins))))
    cmd = ["hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           *flags, os.path.join(REPO, "kubernetriks_amd", "csrc", src), "-o", out_s]
    subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
    try:
        return reachable_divergent_loops(open(out_s).read().split("\n"), kernel)
    finally:
        os.unlink(out_s)


def main():
    args = sys.argv[1:]
    plugins = "--plugins" in args
    flags = [a for a in args if a != "--plugins"]
    fs, loops = compile_and_check(flags, plugins)
    print(json.dumps({"flags": flags, "plugins": plugins, "functions": fs, "divergent_loops": loops}))


if __name__ == "__main__":
    main()
