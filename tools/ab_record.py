#!/usr/bin/env python3
"""Record one A/B gpurun tag as a committed summary (tooling): for every gpurun_out/<tag>/bench*.json
in order, its label, engine build, C3 kernel ms and frac, and the backlog line's kernel ms,
placements/s and node-cache entries read per placement.
Usage: tools/ab_record.py TAG NOTE label0 label1 ... > profiles/<round>_<tag>.json"""
import glob
import json
import os
import sys

tag, note, labels = sys.argv[1], sys.argv[2], sys.argv[3:]
files = sorted(glob.glob(f"gpurun_out/{tag}/bench*.json"), key=lambda f: int(os.path.basename(f)[5:-5] or 0))
rows = []
for i, f in enumerate(files):
    d = json.load(open(f))
    r = d["roofline"]
    row = {"file": f"{tag}/{os.path.basename(f)}", "label": labels[i] if i < len(labels) else "",
           "engine": d["engine"][-12:], "c3_kernel_ms": round(r["kernel_ms_per_launch"], 2), "c3_frac": round(r["frac"], 4),
           "c3_placements_per_s": round(d["value"]),
           "c3_nodes_read_per_placement": round(d["totals"]["nodes_read"] / max(d["totals"]["placements"], 1), 1)}
    bl = d.get("backlog")
    if bl:
        tot = bl["totals"]
        row.update({"backlog_kernel_ms": round(bl["roofline"]["kernel_ms_per_launch"], 2),
                    "backlog_placements_per_s": round(bl["placements_per_s"]),
                    "backlog_nodes_read_per_placement": round(tot["nodes_read"] / max(tot["placements"], 1), 1)})
    rows.append(row)
print(json.dumps({"tag": tag, "note": note, "runs": rows}, indent=1))
