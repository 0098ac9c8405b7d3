#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (CSV output).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of a wide coalesced read, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [--marked]
With --marked, only the dispatches between the first two k_gk_mark launches
count (bench.py's timed region).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirname, counter, marked=False):
    files = glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("gk::", "")
                rows.append((int(row["Dispatch_Id"]), name, float(row["Counter_Value"])))
    rows.sort()
    if marked:
        marks = [d for d, nm, _ in rows if nm.startswith("k_gk_mark")]
        assert len(marks) >= 2, "no k_gk_mark window"
        rows = [r for r in rows if marks[0] < r[0] < marks[1]]
    acc = defaultdict(list)
    for _, name, v in rows:
        acc[name].append(v)
    return acc


def main():
    fdir, wdir, out = sys.argv[1:4]
    marked = "--marked" in sys.argv[4:]
    fetch, write = load(fdir, "FETCH_SIZE", marked), load(wdir, "WRITE_SIZE", marked)
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
        w = sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
        res[k] = {"dispatches": max(len(fetch.get(k, [])), len(write.get(k, []))),
                  "fetch_kib_avg": round(f, 3), "write_kib_avg": round(w, 3),
                  "bytes_per_launch": round((2.0 * f + w) * 1024.0)}
    with open(out, "w") as fh:
        note = "bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH correction"
        if marked:
            note += "; dispatches of bench.py's timed region only (between the k_gk_mark launches)"
        json.dump({"note": note, "kernels": res}, fh, indent=1)
    print(json.dumps(res, indent=1)[:3000])


if __name__ == "__main__":
    main()
