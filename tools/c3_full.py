#!/usr/bin/env python3
"""Full dual (and primal) simplex solves of the dense generator on the GPU:
pivots, wall time, objective, re-inversions; compared with the oracle's
objective when tests/golden/dense_full_<m>x<n>.json exists.
usage: python tools/c3_full.py [M N [meth [tm_lim_ms]]]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
sys.path.insert(0, os.path.join(ROOT, "tests"))
from kkt import dense_kkt  # noqa: E402
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    meth = int(sys.argv[3]) if len(sys.argv) > 3 else gk.GLP_DUAL
    tm = int(sys.argv[4]) if len(sys.argv) > 4 else 120000
    ctx = gk.Context(0)
    prob = problems.gen_dense(m, n, seed=42)
    P = gk.GkProblem(ctx, prob)
    # progress every 2000 pivots (it_lim steps), so a long solve keeps printing
    t0 = time.perf_counter()
    ret = 8
    steps = []
    while ret == 8 and time.perf_counter() - t0 < tm / 1000.0:
        it0, s0 = P.it_cnt, time.perf_counter()
        ret = gk.glp_simplex(P, gk.SMCP(meth=meth, it_lim=2000, msg_lev=gk.GLP_MSG_ERR))
        st = P.stats()
        steps.append({"pivots": P.it_cnt - it0, "seconds": round(time.perf_counter() - s0, 3),
                      "reinversions": st.reinversions, "s_reinvert": round(st.seconds_reinvert, 3),
                      "refinements": st.refinements,
                      "bytes_per_pivot": round(st.bytes_pivots / max(1, st.pivots))})
        print(json.dumps({"it_cnt": P.it_cnt, "ret": ret, **steps[-1]}), flush=True)
    dt = time.perf_counter() - t0
    out = {"m": m, "n": n, "meth": meth, "ret": ret, "obj": P.obj_val, "it_cnt": P.it_cnt,
           "pbs_stat": P.pbs_stat, "dbs_stat": P.dbs_stat, "seconds": round(dt, 3),
           "pivots_per_s": round(P.it_cnt / dt, 1),
           "reinversions": sum(x["reinversions"] for x in steps), "refinements": sum(x["refinements"] for x in steps),
           "s_reinvert": round(sum(x["s_reinvert"] for x in steps), 3),
           "newton_min_k": os.environ.get("GK_NEWTON_MIN_K", "default (512)")}
    if ret == 0:
        out["kkt"] = dense_kkt(P, prob)
    gold = os.path.join(ROOT, "tests", "golden", f"dense_full_{m}x{n}.json")
    if os.path.exists(gold):
        g = json.load(open(gold))
        out["oracle_obj"] = g["obj_val"]
        out["oracle_it_cnt"] = g["it_cnt"]
        out["rel_diff"] = abs(P.obj_val - g["obj_val"]) / max(1.0, abs(g["obj_val"]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
