#!/usr/bin/env python3
"""Static instruction mix of the event-loop pieces (tooling, not product): compiles
tools/probe_isa.hip for gfx950 and counts, per probe kernel, VALU / SALU / LDS / VMEM / SMEM /
branch instructions (lane spills v_writelane/v_readlane and v_readfirstlane listed apart).

Usage: tools/probe_isa.py [extra hipcc flags, e.g. -DK10S_SPLIT=0]"""
import os
import re
import subprocess
import sys
from collections import Counter, OrderedDict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(op):
    if op in ("v_writelane_b32", "v_readlane_b32"):
        return "lanespill"
    if op == "v_readfirstlane_b32":
        return "rfl"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_endpgm", "s_barrier")):
        return "other"
    if op.startswith("s_"):
        return "salu"
    return "other"


def mix(asm_text):
    out = OrderedDict()
    cur = None
    for line in asm_text.splitlines():
        m = re.match(r"^([_A-Za-z][\w$.]*):", line)
        if m and not m.group(1).startswith(".L"):
            cur = m.group(1)
            out.setdefault(cur, Counter())
            continue
        if cur is None:
            continue
        if line.strip().startswith(".end_amdhsa_kernel") or line.startswith("\t.size"):
            cur = None
            continue
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        out[cur][classify(t.split()[0])] += 1
    return out


def main():
    extra = sys.argv[1:] or ["-DK10S_SPLIT=0"]
    asm = "/tmp/probe_isa.s"
    cmd = ["hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           *extra, os.path.join(REPO, "tools", "probe_isa.hip"), "-o", asm]
    subprocess.check_call(cmd)
    res = mix(open(asm).read())
    keys = ["valu", "rfl", "lanespill", "salu", "lds", "vmem", "smem", "branch"]
    print(f"{'kernel':60s} " + " ".join(f"{k:>9s}" for k in keys))
    for name, c in res.items():
        if not name.startswith("_Z"):
            continue
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"\(.*", "", dem)
        print(f"{dem[:60]:60s} " + " ".join(f"{c[k]:9d}" for k in keys))


if __name__ == "__main__":
    main()
