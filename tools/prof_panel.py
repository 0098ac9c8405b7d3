#!/usr/bin/env python3
"""MFMA panel pricing (gk_panel.hip) against the column pass on C3's
HBM-bound regime: the dense generator (default 4096 x 16384, seed 42)
advanced to pivot `start` with the default engine, then alternating windows of
`steps` it_lim=100 calls with GK_PANEL=0 (the column pass over A) and
GK_PANEL=<rows>; pivots/s, panel hits and refills per window, one JSON line
each.  usage: prof_panel.py [start] [steps] [rows] [m n]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    start = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = sys.argv[3] if len(sys.argv) > 3 else "32"
    m = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 16384
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, problems.gen_dense(m, n, seed=42, keep_dense=False))
    adv = gk.SMCP(meth=gk.GLP_DUAL, it_lim=2000, msg_lev=gk.GLP_MSG_ERR)
    t0 = time.perf_counter()
    hits = refills = 0
    while P.it_cnt < start:
        if gk.glp_simplex(P, adv) != 8:
            print(json.dumps({"error": "solved before the window", "it_cnt": P.it_cnt, "obj": P.obj_val}))
            return
        st = P.stats()
        hits += st.panel_hits
        refills += st.panel_refills
        if P.it_cnt % 20000 == 0:
            print(json.dumps({"advance": P.it_cnt, "seconds": round(time.perf_counter() - t0, 2),
                              "hits": hits, "refills": refills}), flush=True)
    print(json.dumps({"advanced_to": P.it_cnt, "seconds": round(time.perf_counter() - t0, 2),
                      "hits": hits, "refills": refills}), flush=True)
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR)
    for mode in ("0", rows, "0", rows):
        os.environ["GK_PANEL"] = mode
        gk.glp_simplex(P, parm)                 # the graphs of this plan
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        piv = h = r = 0
        for _ in range(steps):
            it0 = P.it_cnt
            gk.glp_simplex(P, parm)
            st = P.stats()
            piv += P.it_cnt - it0
            h += st.panel_hits
            r += st.panel_refills
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"panel": int(mode), "from": P.it_cnt - piv, "pivots": piv, "seconds": round(dt, 4),
                          "pivots_per_s": round(piv / dt, 1), "hits": h, "refills": r}), flush=True)


if __name__ == "__main__":
    main()
