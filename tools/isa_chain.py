#!/usr/bin/env python3
"""Dependent-load chains in a kernel's ISA (hipcc --save-temps .s): prints,
in program order up to the first s_barrier (or --all), each vector / scalar
load and each wait that drains loads, so serialised load trips (a load
issued only after a wait for the previous one) are visible.

usage: isa_chain.py FILE.s KERNEL_SUBSTRING [--all]"""
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    allb = "--all" in sys.argv
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l))
    trips, pend = 0, 0
    for l in lines[start + 1:]:
        if "s_endpgm" in l or (not allb and "s_barrier" in l):
            print("   ", l.strip())
            break
        t = l.strip()
        if re.match(r"(global|buffer|flat)_load|s_load|s_buffer_load", t):
            pend += 1
            print(f"  L {t[:70]}")
        elif t.startswith("s_waitcnt") and ("vmcnt(0)" in t or "lgkmcnt(0)" in t):
            if pend:
                trips += 1
                print(f"W{trips:3d} {t}   ({pend} loads since last drain)")
            pend = 0
        elif t.startswith("s_cbranch") or t.startswith(".LBB"):
            print(f"    {t[:60]}")
    print("drains:", trips)


if __name__ == "__main__":
    main()
