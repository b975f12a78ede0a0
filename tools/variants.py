#!/usr/bin/env python3
"""Build semantics-neutral variant libraries for A/B runs on the GPU (load one with K10S_LIB=...).

Live knobs (round 4 removed the measured-and-not-kept alternatives; their A/B history is DESIGN §7c):
  tooling   prof  -DK10S_PROF=1 (cycle attribution, bench.py --profile); EXEC_CHECK=1|2|3 (entry guards /
            loop bounds, tools/launch_trace.py); BEACON=1 (host-mapped progress beacon,
            tools/beacon_trace.py); WALL=1 (tools/wall_spread.py)
  numeric   wN -DK10S_WAVES_PER_EU=N; sN -DK10S_SPLIT=N (out-of-line handlers); pN -DK10S_SCAN_PIPE=N
            (unit-surface scan loads N steps ahead); LOOP_SCAN_PIPE=N; qN -DK10S_FQW=N (FIFO window
            entries in LDS); hN -DK10S_HEAP_D=N (event-heap arity 8/16/32/64); AQ_TOP=N;
            FAIR_SHIFT=N, FAIR_BAND=N (wave priorities)
  round 5   WINDOWS=0|1, WIN_NOTSCHED=0|1, FUSE_FINISH=0|1, RUNS=0|1 (events handled together);
            SEC_SGPR=0|1 (section bases from the LDS table / from the workgroup id); TILE_BEST=1,
            TILE_ALWAYS=1 (best-node tiles, measured and not kept)
  round 6   TILE_PRUNE=0|1 (block-bound scans of a tile's fitting pods), AQ_SORTED=0|1 (sorted-mode action
            queue and bulk move-all appends)
  NAME=v    -DK10S_NAME=v (any of the above by name), parts joined by '+'
Usage: tools/variants.py prof w8 s1 WAVES_PER_EU=8+FQW=4 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetriks_amd.build import REPO, build  # noqa: E402


def flags(name):
    out = []
    for part in name.split("+"):
        if "=" in part:                      # any engine knob: NAME=value -> -DK10S_NAME=value
            out.append(f"-DK10S_{part}")
        elif part == "prof":
            out.append("-DK10S_PROF=1")
        elif part.startswith("w"):
            out.append(f"-DK10S_WAVES_PER_EU={int(part[1:])}")
        elif part.startswith("p"):
            out.append(f"-DK10S_SCAN_PIPE={int(part[1:])}")
        elif part.startswith("q"):
            out.append(f"-DK10S_FQW={int(part[1:])}")
        elif part.startswith("h") and part[1:].isdigit():
            out.append(f"-DK10S_HEAP_D={int(part[1:])}")
        elif part.startswith("s"):
            out.append(f"-DK10S_SPLIT={int(part[1:])}")
        else:
            raise SystemExit(f"unknown variant part {part}")
    return out


if __name__ == "__main__":
    for v in sys.argv[1:]:
        tag = v.replace("=", "").replace("+", "_")
        print(build(force=True, extra=flags(v), out=os.path.join(REPO, "build", f"libk10s_{tag}.so")))
