#!/usr/bin/env python3
"""C3 primal simplex in it_lim steps (the bench's c3_primal_steps leg), with
each step's time and pivots: python tools/primal_steps.py [M N [STEPS [IT_LIM]]]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    it_lim = int(sys.argv[4]) if len(sys.argv) > 4 else 100
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, problems.gen_dense(m, n, seed=42))
    parm = gk.SMCP(meth=gk.GLP_PRIMAL, it_lim=it_lim, msg_lev=gk.GLP_MSG_ERR)
    for k in range(steps):
        it0, t0 = P.it_cnt, time.perf_counter()
        ret = gk.glp_simplex(P, parm)
        dt = time.perf_counter() - t0
        st = P.stats()
        print(json.dumps({"step": k, "ret": ret, "pivots": P.it_cnt - it0, "ms": round(1e3 * dt, 3),
                          "pivots_per_s": round((P.it_cnt - it0) / dt, 1), "batches": st.batches,
                          "reinversions": st.reinversions, "ms_batches": round(1e3 * st.seconds_batches, 3),
                          "ms_eval": round(1e3 * st.seconds_eval, 3)}), flush=True)


if __name__ == "__main__":
    main()
