#!/usr/bin/env python3
"""Static instruction mix per device function of the event-loop kernel (tooling, not product):
compiles kubernetriks_amd/csrc/k10s_kernels.hip for gfx950 (extra hipcc flags from the command
line, e.g. -DK10S_SPLIT=1) and counts, per function (the run kernel, each out-of-line handler, the
scheduling cycle), VALU / v_readfirstlane / lane spills (v_writelane, v_readlane) / SALU / LDS /
VMEM / SMEM / scratch instructions, plus the function's VGPR count and scratch bytes.  Static
counts: a proxy for the per-event cost of the handlers (the per-kind dynamic cost is the K10S_PROF
cycle attribution, bench.py --profile).  Prints one JSON object."""
import json
import os
import re
import subprocess
import sys
from collections import OrderedDict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
from probe_isa import classify  # noqa: E402


def main():
    out_s = "/tmp/k10s_isa_functions.s"
    cmd = ["hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only", "-S",
           *sys.argv[1:], os.path.join(REPO, "kubernetriks_amd", "csrc", "k10s_kernels.hip"), "-o", out_s]
    subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
    funcs = OrderedDict()
    cur = None
    for line in open(out_s):
        m = re.match(r"^([_A-Za-z][_A-Za-z0-9]*):", line)
        if m and not m.group(1).startswith(".L"):
            cur = m.group(1)
            funcs[cur] = {"valu": 0, "rfl": 0, "lanespill": 0, "salu": 0, "lds": 0, "vmem": 0, "smem": 0, "branch": 0,
                          "scratch": 0}
            continue
        if cur is None:
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        t = line.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        k = classify(op)
        if op.startswith("scratch_"):
            funcs[cur]["scratch"] += 1
        if k in funcs[cur]:
            funcs[cur][k] += 1
    stats = {}
    fn = None
    for line in open(out_s):
        m = re.match(r"^([_A-Za-z][_A-Za-z0-9]*):", line)
        if m and not m.group(1).startswith(".L"):
            fn = m.group(1)
        m = re.search(r"; NumVgprs: (\d+)", line)
        if m and fn in funcs:
            stats.setdefault(fn, {})["vgprs"] = int(m.group(1))
        m = re.search(r"; ScratchSize: (\d+)", line)
        if m and fn in funcs:
            stats.setdefault(fn, {})["scratch_bytes"] = int(m.group(1))
    keep = {}
    for name, c in funcs.items():
        if sum(c.values()) == 0:
            continue
        short = re.sub(r"^_ZN4k10s\d+", "", name)
        short = re.sub(r"^_Z\d+", "", short)
        keep[short[:48]] = dict(c, **stats.get(name, {}))
    print(json.dumps({"flags": sys.argv[1:], "functions": keep}, indent=1))


if __name__ == "__main__":
    main()
