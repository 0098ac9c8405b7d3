#!/usr/bin/env python3
"""Symbolise the GK_HOST_PROF lines of a log ("[gk hostprof] <n> 0x<offset>")
against the library build they came from, summed per function.
usage: symbolize_hostprof.py LOG [LIB]"""
import collections
import re
import subprocess
import sys

log = sys.argv[1]
lib = sys.argv[2] if len(sys.argv) > 2 else "glpk.js_amd/libglpk_mi355x.so"
runs, cur = [], None
for line in open(log):
    if "[gk hostprof]" not in line:
        continue
    m = re.search(r"\] (\d+) samples, (\d+) outside", line)
    if m:
        cur = {"total": int(m.group(1)), "other": int(m.group(2)), "pcs": []}
        runs.append(cur)
        continue
    m = re.search(r"\] (\d+) 0x([0-9a-f]+)", line)
    if m and cur is not None:
        cur["pcs"].append((int(m.group(1)), int(m.group(2), 16)))
for r in runs:
    addrs = "\n".join(hex(a) for _, a in r["pcs"]) + "\n"
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-symbolizer", "--obj=" + lib, "--no-inlines", "-C",
                          "--output-style=GNU"], input=addrs, capture_output=True, text=True).stdout.split("\n")
    names = [out[2 * i] for i in range(len(r["pcs"]))]
    agg = collections.Counter()
    for (n, _), nm in zip(r["pcs"], names):
        agg[nm.split("(")[0][:110]] += n
    print(f"== {r['total']} samples ({r['other']} outside the library; top offsets only below)")
    for nm, n in agg.most_common(25):
        print(f"{n:7d} {100.0 * n / max(1, r['total']):5.1f}%  {nm}")
