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

Usage: tools/divergent_loops.py [--plugins] [hipcc flags...]"""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "_Z15k10s_run_kerneljiddmPj"


def divergent_loops(asm_lines, kernel=KERNEL):
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
        inner = any("Inner Loop Header" in x for x in comment)
        swappc = sum("s_swappc_b64" in l for l in body)
        # allowed: an innermost loop that calls nothing (lane-strided copies and scans)
        out.append({"line": i - st, "header": hdr, "comment": " | ".join(comment), "blocks_lines": len(body),
                    "swappc": swappc, "ok": inner and swappc == 0})
    return out


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
        return divergent_loops(open(out_s).read().split("\n"), kernel)
    finally:
        os.unlink(out_s)


def main():
    args = sys.argv[1:]
    plugins = "--plugins" in args
    flags = [a for a in args if a != "--plugins"]
    print(json.dumps({"flags": flags, "plugins": plugins, "divergent_loops": compile_and_check(flags, plugins)}))


if __name__ == "__main__":
    main()
