#!/usr/bin/env python3
"""Summarize the bench lines of one gpurun tag (tooling): for every gpurun_out/<tag>/bench*.json,
engine build, workload, placements/s, kernel ms, roofline frac.  Usage: tools/ab_summary.py TAG [labels...]"""
import glob
import json
import os
import sys

tag = sys.argv[1]
labels = sys.argv[2:]
files = sorted(glob.glob(f"gpurun_out/{tag}/bench*.json"), key=lambda f: int(os.path.basename(f)[5:-5] or 0))
for i, f in enumerate(files):
    try:
        d = json.load(open(f))
    except Exception as ex:
        print(f, "unreadable", ex)
        continue
    r = d["roofline"]
    lab = labels[i] if i < len(labels) else ""
    print(f"{os.path.basename(f):12s} {lab:10s} {d['config'].get('workload_name', ''):11s} {d['value']/1e6:8.2f} M/s "
          f"kernel {r['kernel_ms_per_launch']:8.1f} ms frac {r['frac']:.3f}  {d['engine'][-12:]}")
