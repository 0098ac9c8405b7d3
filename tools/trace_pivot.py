#!/usr/bin/env python3
"""Per-block timeline of one dual pivot on C3 (gk_bfd_profile(2)): for each
pivot kernel, the dispatch ramp (first to last block entry), the execution
span (first entry to last exit) and the per-block durations, averaged over
a number of traced pivots.  Eager launches (profiling disables graphs)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402

NAMES = ["top", "row", "ratio", "ftran1", "commit", "trow_finish", "ftran_split", "ftran_reduce"]


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, problems.gen_dense(m, n, seed=42))
    assert P.factorize() == 0
    gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=warm, msg_lev=gk.GLP_MSG_ERR))
    # GK_TRACE_GRAPH=1: stamps inside the replayed graphs (gk_bfd_profile 3)
    P.profile(3 if os.environ.get("GK_TRACE_GRAPH") else 2)
    khz = 100000.0
    acc = {}
    ph = {}
    slow = {}
    ph0 = {}
    reps = 20
    for _ in range(reps):
        gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=60, msg_lev=gk.GLP_MSG_ERR))
        tr = P.trace().astype(np.int64)
        t_ref = None
        for k, name in enumerate(NAMES):
            e = tr[k, :, 0]
            x = tr[k, :, 1]
            if e[0] == 0:
                continue
            t0 = e[0]
            valid = (e >= t0 - 10) & (e > 0) & (x >= e)
            # blocks of this pivot: entries within 1 ms of block 0's
            valid &= np.abs(e - t0) < khz
            ev, xv = e[valid], x[valid]
            if t_ref is None:
                t_ref = ev.min()
            p0 = 8 * 2048 * 2
            phs = P.trace_raw[p0 + k * 2048 * 8: p0 + (k + 1) * 2048 * 8].reshape(2048, 8).astype(np.int64)
            sel = np.where(valid)[0]
            rel = phs[sel] - e[sel][:, None]
            rel[(phs[sel] == 0) | (rel < 0) | (rel > khz)] = 0
            if rel.any():
                cnt = np.maximum((rel > 0).sum(axis=0), 1)
                ph.setdefault(name, []).append(rel.sum(axis=0) / cnt)
                ph0.setdefault(name, []).append(rel[0])
            sl = slow.setdefault(name, np.zeros((2, len(e))))
            sl[0, sel] += (x[sel] - t0) / reps
            sl[1, sel] += (e[sel] - t0) / reps
            a = acc.setdefault(name, [])
            a.append(((ev.min() - t_ref), ev.max() - ev.min(), xv.max() - ev.min(), np.mean(xv - ev),
                      np.max(xv - ev), valid.sum()))
    print("phase stamps of wave 0, us after block entry (mean over blocks and calls):")
    for k, name in enumerate(NAMES):
        if name in ph and ph[name]:
            a = np.array(ph[name], dtype=float).mean(axis=0)
            print(f"  {name:14s} " + " ".join(f"{v/100:6.2f}" for v in a if v > 0))
            a0 = np.array(ph0[name], dtype=float).mean(axis=0)
            print(f"  {name + ' b0':14s} " + " ".join(f"{v/100:6.2f}" for v in a0))
    print(f"C3 {m}x{n}, last pivot of {reps} calls of 60 pivots after {warm} (times in us; device clock 100 MHz)")
    print(f"{'kernel':14s} {'start':>8s} {'ramp':>7s} {'span':>7s} {'blk avg':>8s} {'blk max':>8s} {'blocks':>7s}")
    print("latest-finishing blocks (exit and entry after block 0's entry, us, mean over calls):")
    for name, sl in slow.items():
        o = np.argsort(-sl[0])[:6]
        print(f"  {name:14s} " + " ".join(f"b{b}:{sl[0, b]/100:.2f}(in {sl[1, b]/100:.2f})" for b in o))
    for name, a in acc.items():
        a = np.array(a, dtype=float)
        mu = a.mean(axis=0)
        print(f"{name:14s} {mu[0]/100:8.2f} {mu[1]/100:7.2f} {mu[2]/100:7.2f} {mu[3]/100:8.2f} {mu[4]/100:8.2f} {mu[5]:7.0f}")


if __name__ == "__main__":
    main()
