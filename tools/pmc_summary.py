#!/usr/bin/env python3
"""Summarize two rocprofv3 --pmc passes of one kernel into HBM-side bytes per launch (tooling).

Reads come from the L2's memory-side read requests by size (gfx950: TCC_EA0_RDREQ_32B/_64B/_128B,
summed over the TCC instances): 32·n32 + 64·n64 + 128·n128 bytes.  This is exact where FETCH_SIZE
is not: FETCH_SIZE = TCC_EA0_RDREQ × 64 B on gfx950 (MI355X_MICROARCH.md, HBM section), which is
half the bytes of the 128-B requests that wide streaming reads make, and the right count for
64-B ones.  Round 4's doubling of FETCH_SIZE over-counted the 64-B share.  Writes come from
TCC_EA0_WRREQ (64-B ones counted by _64B, the rest 32 B): WRITE_SIZE's own formula.  Infinity
Cache hits are counted, not excluded (no counter separates them).
Usage: pmc_summary.py RD_DIR WR_DIR KERNEL BENCH_JSON
  RD_DIR: a pass of TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum,TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum
  WR_DIR: a pass of TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum (and optionally the _DRAM ones)
  BENCH_JSON: the bench line printed during the RD pass; it names the engine build, the config and
  the scan mode, which bench.py matches before it reports `traffic`."""
import csv
import glob
import json
import os
import sys


def per_launch(d, kernel):
    vals, n = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Kernel_Name"].startswith(kernel):
                c = row["Counter_Name"]
                vals[c] = vals.get(c, 0.0) + float(row["Counter_Value"])
                n.setdefault(c, set()).add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    return {c: v / max(1, len(n[c])) for c, v in vals.items()}, max((len(s) for s in n.values()), default=0)


def main():
    rdir, wdir, kernel, bench_json = sys.argv[1:5]
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    cfg = b["config"]
    r, nr = per_launch(rdir, kernel)
    w, nw = per_launch(wdir, kernel)
    rd = 32.0 * r["TCC_EA0_RDREQ_32B_sum"] + 64.0 * r["TCC_EA0_RDREQ_64B_sum"] + 128.0 * r["TCC_EA0_RDREQ_128B_sum"]
    wr = 64.0 * w["TCC_EA0_WRREQ_64B_sum"] + 32.0 * (w["TCC_EA0_WRREQ_sum"] - w["TCC_EA0_WRREQ_64B_sum"])
    out = {
        "method": "rocprofv3 --kernel-trace --pmc, two passes over one bench launch: reads = 32/64/128 B x "
                  "TCC_EA0_RDREQ_32B/_64B/_128B (exact request sizes; FETCH_SIZE tallies every request at 64 B), "
                  "writes = WRITE_SIZE's formula from TCC_EA0_WRREQ and _64B; per dispatch",
        "kernel": kernel, "config": [cfg["replicas_per_gpu"], cfg["nodes"], cfg["pods_per_replica"]],
        "workload": cfg.get("workload_name", "c3"), "launches": [nr, nw],
        "engine": b.get("engine"), "scan_mode": b.get("roofline", {}).get("scan_mode", "full"),
        "score_plugins": cfg.get("score_plugins", "least"),
        "read_requests": {k: r.get(k) for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
                                                "TCC_EA0_RDREQ_128B_sum")},
        "write_requests": {k: v for k, v in w.items()},
        "read_bytes": rd, "write_bytes": wr,
        "fetch_size_equivalent_kib": r["TCC_EA0_RDREQ_sum"] * 64.0 / 1024.0,
        "hbm_bytes_per_launch": rd + wr,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
