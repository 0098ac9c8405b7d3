#!/usr/bin/env python3
"""Where the dual simplex reports numerical instability on C3: the dense
generator (default 4096 x 16384, seed 42) advanced from the slack basis in
it_lim=2000 calls (the bench's c3_mid advance) up to `target` pivots; one JSON
line per call with the engine's counters, the report lines of the call on
stderr.  Run once per GK_PANEL / GK_PANEL_AGE setting (read once per process).
usage: instab_probe.py [target] [m n]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    target = int(sys.argv[1]) if len(sys.argv) > 1 else 60000
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, problems.gen_dense(m, n, seed=42, keep_dense=False))
    adv = gk.SMCP(meth=gk.GLP_DUAL, it_lim=2000, msg_lev=gk.GLP_MSG_ERR)
    t0 = time.perf_counter()
    env = {k: os.environ.get(k) for k in ("GK_PANEL", "GK_PANEL_AGE")}
    while P.it_cnt < target:
        it0 = P.it_cnt
        print(f"--- call from it_cnt={it0}", file=sys.stderr, flush=True)
        ret = gk.glp_simplex(P, adv)
        st = P.stats()
        print(json.dumps({"env": env, "from": it0, "to": P.it_cnt, "ret": ret, "obj": P.obj_val,
                          "hits": st.panel_hits, "refills": st.panel_refills,
                          "t": round(time.perf_counter() - t0, 2)}), flush=True)
        if ret != 8:
            break


if __name__ == "__main__":
    main()
