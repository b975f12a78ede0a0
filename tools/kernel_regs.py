#!/usr/bin/env python3
"""Per-kernel register/scratch summary of a gfx950 assembly file (tooling): name, VGPRs, SGPRs,
VGPR/SGPR spills, scratch bytes.  Usage: tools/kernel_regs.py file.s"""
import re
import sys

text = open(sys.argv[1]).read()
meta = text[text.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    get = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, blk) or [None, "?"])[1]
    print(f"{get('name')[:40]:40s} vgpr={get('vgpr_count'):>4} sgpr={get('sgpr_count'):>4} "
          f"vspill={get('vgpr_spill_count'):>4} sspill={get('sgpr_spill_count'):>4} scratch={get('private_segment_fixed_size')}")
