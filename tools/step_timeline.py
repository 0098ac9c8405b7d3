#!/usr/bin/env python3
"""Timeline of one bench step from a rocprofv3 results database
(`rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o run -- python3
bench.py ...`): every kernel and copy of the step with its start offset,
duration and the idle gap before it (host work shows up as gaps), the pivot
kernels of a batch collapsed into one line.  Steps are delimited by the
per-call upload kernel (k_scatter_segments) inside bench.py's marked region.

usage: step_timeline.py DB [--step I]"""
import argparse
import sqlite3

PIVOT = ("k_dual_row", "k_dual_ratio", "k_dual_update", "k_dual_ftran1", "k_dual_commit", "k_dual_col")


def short(nm):
    return nm.split("(")[0].replace("void ", "").replace("gk::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=-2)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ev = [(s, e - s, short(n)) for n, s, e in c.execute("select name, start, end from kernels")]
    try:
        for s, e, src, dst in c.execute("select start, end, src_agent_type, dst_agent_type from memory_copies"):
            ev.append((s, e - s, f"copy {src}->{dst}"))
    except sqlite3.Error:
        try:
            for s, e in c.execute("select start, end from memory_copies"):
                ev.append((s, e - s, "copy"))
        except sqlite3.Error:
            pass
    ev.sort()
    marks = [s for s, _, n in ev if n.startswith("k_gk_mark")]
    ev = [x for x in ev if marks[0] < x[0] < marks[1]]
    starts = [i for i, x in enumerate(ev) if x[2] == "k_scatter_segments"]
    starts.append(len(ev))
    k = a.step if a.step >= 0 else len(starts) - 1 + a.step
    sel = ev[starts[k]:starts[k + 1]]
    t0 = sel[0][0]
    prev_end = t0
    gap_tot = busy = 0.0
    i = 0
    print(f"step {k} of {len(starts) - 1}: {(sel[-1][0] + sel[-1][1] - t0) / 1e3:.1f} us from the upload kernel "
          f"to the last event")
    while i < len(sel):
        s, d, n = sel[i]
        gap = max(0, s - prev_end)
        if n.startswith(PIVOT):
            j = i
            while j < len(sel) and sel[j][2].startswith(PIVOT):
                j += 1
            end = max(x[0] + x[1] for x in sel[i:j])
            kb = sum(x[1] for x in sel[i:j])
            print(f"{(s - t0) / 1e3:9.1f} {gap / 1e3:7.1f} gap  batch of {j - i} pivot kernels: span "
                  f"{(end - s) / 1e3:.1f} us, kernel time {kb / 1e3:.1f} us")
            busy += kb
            gap_tot += gap
            prev_end = end
            i = j
            continue
        print(f"{(s - t0) / 1e3:9.1f} {gap / 1e3:7.1f} gap  {d / 1e3:7.1f} us  {n[:60]}")
        gap_tot += gap
        busy += d
        prev_end = max(prev_end, s + d)
        i += 1
    print(f"gaps {gap_tot / 1e3:.1f} us, busy {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
