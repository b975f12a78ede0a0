#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes for one kernel into HBM bytes per launch.

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch.  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM
section) gfx950's FETCH_SIZE reports half of the bytes of wide coalesced streaming reads, so it is
doubled; WRITE_SIZE is taken as read.  Usage: pmc_summary.py FETCH_DIR WRITE_DIR KERNEL BENCH_JSON
(BENCH_JSON: the bench line printed during the FETCH pass; it names the engine build, the config and
the scan mode, which bench.py matches before it reports `traffic`)."""
import csv
import json
import sys


def per_launch(path, kernel, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and row["Kernel_Name"].startswith(kernel):
                vals.append(float(row["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    fdir, wdir, kernel, bench_json = sys.argv[1:5]
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    cfg = b["config"]
    config = json.dumps([cfg["replicas_per_gpu"], cfg["nodes"], cfg["pods_per_replica"]])
    fk, nf = per_launch(f"{fdir}/run_counter_collection.csv", kernel, "FETCH_SIZE")
    wk, nw = per_launch(f"{wdir}/run_counter_collection.csv", kernel, "WRITE_SIZE")
    out = {
        "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over one bench "
                  "step; values in KiB per dispatch; FETCH_SIZE doubled (gfx950 reports half of 16-B/lane streaming "
                  "reads, MI355X_MICROARCH.md HBM section); WRITE_SIZE as read",
        "kernel": kernel, "config": json.loads(config), "workload": cfg.get("workload_name", "c3"),
        "launches": [nf, nw],
        "engine": b.get("engine"), "scan_mode": b.get("roofline", {}).get("scan_mode", "full"),
        "score_plugins": cfg.get("score_plugins", "least"),
        "fetch_size_kib": fk, "write_size_kib": wk,
        "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0 if fk is not None and wk is not None else None,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
