#!/usr/bin/env python3
"""Microbenchmark of the scheduling scan alone (k10s_schedule_one_batch); see
kubernetriks_amd/scanbench.py.  Prints one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=8192)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from kubernetriks_amd.scanbench import measure
    print(json.dumps(measure(a.problems, a.nodes, a.iters)))


if __name__ == "__main__":
    main()
