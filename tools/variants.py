#!/usr/bin/env python3
"""Build semantics-neutral variant libraries for A/B runs on the GPU (load one with K10S_LIB=...).

  prof   -DK10S_PROF=1: cycle attribution of the event loop (bench.py --profile)
  wN     -DK10S_WAVES_PER_EU=N
  sN     -DK10S_SPLIT=N
  pN     -DK10S_SCAN_PIPE=N (scan loads N steps ahead)
  qN     -DK10S_FQW=N (delay-class FIFO window entries in LDS)
  bfN    -DK10S_SCAN_BF=N (branch-free node scan)
Usage: tools/variants.py prof w8 s1 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubernetriks_amd.build import REPO, build  # noqa: E402


def flags(name):
    out = []
    for part in name.split("_"):
        if part == "prof":
            out.append("-DK10S_PROF=1")
        elif part.startswith("w"):
            out.append(f"-DK10S_WAVES_PER_EU={int(part[1:])}")
        elif part.startswith("p"):
            out.append(f"-DK10S_SCAN_PIPE={int(part[1:])}")
        elif part.startswith("q"):
            out.append(f"-DK10S_FQW={int(part[1:])}")
        elif part.startswith("bf"):
            out.append(f"-DK10S_SCAN_BF={int(part[2:])}")
        elif part.startswith("s"):
            out.append(f"-DK10S_SPLIT={int(part[1:])}")
        else:
            raise SystemExit(f"unknown variant part {part}")
    return out


if __name__ == "__main__":
    for v in sys.argv[1:]:
        print(build(force=True, extra=flags(v), out=os.path.join(REPO, "build", f"libk10s_{v}.so")))
