#!/usr/bin/env python3
"""Derived occupancy / LDS / L2 / issue figures for one kernel from several rocprofv3 --pmc passes
(tooling).  Usage: pmc_derive.py KERNEL BENCH_JSON DIR [DIR ...]
Each DIR holds one pass's run_counter_collection.csv (and run_kernel_trace.csv when present);
counters are summed over the kernel's dispatches.  Units per MI355X_MICROARCH.md: SQ_WAVE_CYCLES and
the SQ_WAIT_* / SQ_ACTIVE_INST_* counters count quad-cycles; GRBM_GUI_ACTIVE is summed over the
8 XCDs.  BENCH_JSON: the bench line of one of the passes (events per launch, engine build)."""
import csv
import glob
import json
import os
import sys


def main():
    kernel, bench_json, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    launches = max(1, b["steps"] + b["warmup"])
    events = b["totals"]["events"] / max(1, b["steps"]) if b.get("totals") else None
    ctr, seen, ns = {}, {}, []
    for d in dirs:
        mine = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if row["Kernel_Name"].startswith(kernel):
                    mine[row["Counter_Name"]] = mine.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
        for k, v in mine.items():   # a counter taken in several passes: their mean
            ctr[k] = ctr.get(k, 0.0) + v
            seen[k] = seen.get(k, 0) + 1
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if row["Kernel_Name"].startswith(kernel):
                    ns.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    per = {k: v / seen[k] / launches for k, v in ctr.items()}   # per launch
    kns = sum(ns) / len(ns) if ns else None
    der = {}
    g = per.get("GRBM_GUI_ACTIVE")
    if g and kns:
        cyc = g / 8.0
        der["effective_clock_GHz"] = cyc / kns
        if "SQ_WAVE_CYCLES" in per:
            der["mean_resident_waves_per_SIMD"] = per["SQ_WAVE_CYCLES"] * 4.0 / (cyc * 1024.0)
        if "SQ_INSTS_VALU" in per:
            der["valu_busy_fraction_at_4_cycles"] = per["SQ_INSTS_VALU"] * 4.0 / (cyc * 1024.0)
    w = per.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
            if k in per:
                der[k.lower() + "_share_of_wave_cycles"] = per[k] / w
    if per.get("SQ_LDS_IDX_ACTIVE"):
        der["lds_bank_conflict_rate"] = per.get("SQ_LDS_BANK_CONFLICT", 0.0) / per["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in per and "TCC_MISS_sum" in per:
        der["l2_hit_rate"] = per["TCC_HIT_sum"] / (per["TCC_HIT_sum"] + per["TCC_MISS_sum"])
    if per.get("TCC_EA0_RDREQ_sum"):
        # memory-side read requests of the L2 that target DRAM (HBM or the Infinity Cache in front of
        # it: the MALL sits on the memory side, so the L2 counters cannot split its hits from HBM)
        der["dram_share_of_l2_read_requests"] = per.get("TCC_EA0_RDREQ_DRAM_sum", 0.0) / per["TCC_EA0_RDREQ_sum"]
    if "TCC_EA0_RDREQ_128B_sum" in per:   # exact request sizes (tools/pmc_summary.py; round 5)
        der["memory_read_bytes"] = (32.0 * per.get("TCC_EA0_RDREQ_32B_sum", 0.0) + 64.0 * per.get("TCC_EA0_RDREQ_64B_sum", 0.0)
                                    + 128.0 * per["TCC_EA0_RDREQ_128B_sum"])
    elif "FETCH_SIZE" in per:
        der["memory_read_bytes"] = 2.0 * per["FETCH_SIZE"] * 1024.0   # round 4: FETCH_SIZE doubled
    if "TCC_EA0_WRREQ_64B_sum" in per and "TCC_EA0_WRREQ_sum" in per:
        der["memory_write_bytes"] = 64.0 * per["TCC_EA0_WRREQ_64B_sum"] + 32.0 * (per["TCC_EA0_WRREQ_sum"] - per["TCC_EA0_WRREQ_64B_sum"])
    elif "WRITE_SIZE" in per:
        der["memory_write_bytes"] = per["WRITE_SIZE"] * 1024.0
    if "memory_read_bytes" in der and "memory_write_bytes" in der and kns:
        tot = der["memory_read_bytes"] + der["memory_write_bytes"]
        der["memory_bytes_per_launch"] = tot
        der["memory_TBps"] = tot / kns / 1e3
        der["memory_frac_of_8TBps"] = tot / kns / 8e3
        if events:
            der["memory_bytes_per_event"] = tot / events
    if "SQ_INSTS_VMEM" in per and events:
        der["vmem_insts_per_event"] = per["SQ_INSTS_VMEM"] / events
    if events:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
            if k in per:
                der[k[9:].lower() + "_insts_per_event"] = per[k] / events
        der["events_per_launch"] = events
    print(json.dumps({"method": "rocprofv3 --kernel-trace --pmc, one pass per counter group over the same bench "
                                "command; counters summed over the kernel's dispatches, divided by the launches",
                      "engine": b.get("engine"), "kernel": kernel, "config": b.get("config"),
                      "kernel_ns": kns, "counters_per_launch": per, "derived": der}, indent=1))


if __name__ == "__main__":
    main()
