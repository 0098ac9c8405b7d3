#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 results database (the default
rocpd SQLite output of `rocprofv3 --kernel-trace --stats -d DIR -o run`).

usage: prof_stats.py DB [--csv OUT] [--grid]
Prints name, calls, total/avg/min/max ns (as rocprofv3's kernel_stats.csv),
and with --grid the grid sizes seen per kernel."""
import argparse
import csv
import sqlite3
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--grid", action="store_true")
    ap.add_argument("--marked", action="store_true",
                    help="only the kernels between the first two k_gk_mark launches (bench.py's timed region)")
    ap.add_argument("--window", type=int, default=0,
                    help="with --marked: the i-th pair of k_gk_mark launches (0-based)")
    ap.add_argument("--json", help="write {kernel: {calls, avg_ns}} of the selection")
    ap.add_argument("--gaps", help="write the idle time between consecutive kernels, per (previous, next) pair")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, workgroup_x, start from kernels order by start").fetchall()
    if a.marked:
        marks = [r[4] for r in rows if r[0].startswith("k_gk_mark")]
        w = 2 * a.window
        assert len(marks) >= w + 2, "no such k_gk_mark window in the trace"
        rows = [r for r in rows if marks[w] < r[4] < marks[w + 1]]
    if a.gaps:
        # end of kernel i to start of kernel i + 1 (one stream: the engine's)
        short = lambda nm: nm.split("(")[0].replace("void ", "").replace("gk::", "")[:40]
        pairs = {}
        for r0, r1 in zip(rows, rows[1:]):
            g = r1[4] - (r0[4] + r0[1])
            if 0 <= g < 200000:           # within one graph / batch (< 200 us)
                pairs.setdefault((short(r0[0]), short(r1[0])), []).append(g)
        with open(a.gaps, "w") as f:
            f.write(f"{'previous':40s} {'next':40s} {'count':>7s} {'median_us':>9s} {'mean_us':>8s} {'p10_us':>7s} {'p90_us':>7s}\n")
            for (k0, k1), v in sorted(pairs.items(), key=lambda kv: -len(kv[1])):
                v = sorted(v)
                q = lambda f_: v[min(len(v) - 1, int(f_ * len(v)))] / 1000
                f.write(f"{k0:40s} {k1:40s} {len(v):7d} {q(0.5):9.2f} {sum(v)/len(v)/1000:8.2f} {q(0.1):7.2f} {q(0.9):7.2f}\n")
    by = {}
    for name, dur, gx, wx, _ in rows:
        e = by.setdefault(name, {"d": [], "grids": set()})
        e["d"].append(dur)
        e["grids"].add(gx // max(1, wx))
    tot = sum(sum(e["d"]) for e in by.values())
    out = []
    for name, e in sorted(by.items(), key=lambda kv: -sum(kv[1]["d"])):
        d = e["d"]
        out.append([name, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / tot, min(d), max(d),
                    statistics.pstdev(d)])
    if a.json:
        import json
        short = lambda nm: nm.split("(")[0].replace("void ", "").replace("gk::", "")
        json.dump({short(r[0]): {"calls": r[1], "avg_ns": round(r[3], 1)} for r in out}, open(a.json, "w"), indent=1)
    w = csv.writer(open(a.csv, "w", newline="") if a.csv else sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for r in out:
        w.writerow(r)
    if a.csv or a.grid:
        for name, e in sorted(by.items(), key=lambda kv: -sum(kv[1]["d"])):
            d = e["d"]
            g = sorted(e["grids"])
            print(f"{name[:70]:70s} {len(d):7d} {sum(d)/len(d)/1000:8.2f} us  blocks {g[:6]}{'...' if len(g) > 6 else ''}")


if __name__ == "__main__":
    main()
