#!/usr/bin/env python3
"""C3 dual mid-solve window: advance the solve to WARM pivots from the slack
basis (it_lim steps of 2000), then run STEPS steps of 100 pivots between two
gk_ctx_mark launches (the rocprofv3 window); prints the engine's bytes per
pivot and the pivots/s of the window.
usage: python tools/c3_mid.py [WARM [STEPS]]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, problems.gen_dense(4096, 16384, seed=42))
    t_adv = time.perf_counter()
    adv = {"reinversions": 0, "refinements": 0, "s_reinvert": 0.0}
    while P.it_cnt < warm:
        ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=min(2000, warm - P.it_cnt),
                                        msg_lev=gk.GLP_MSG_ERR))
        s = P.stats()
        adv["reinversions"] += s.reinversions
        adv["refinements"] += s.refinements
        adv["s_reinvert"] += s.seconds_reinvert
        print(json.dumps({"it_cnt": P.it_cnt}), flush=True)
        assert ret == 8
    t_adv = time.perf_counter() - t_adv
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR)
    gk.glp_simplex(P, parm)
    torch.cuda.synchronize()
    ctx.mark(1)
    t0 = time.perf_counter()
    piv, byts, split = 0, 0.0, {"init": 0.0, "eval": 0.0, "batches": 0.0, "reinvert": 0.0}
    reinv = {"reinversions": 0, "refine_tries": 0, "refinements": 0, "refine_steps": 0, "refine_resid_max": 0.0}
    for _ in range(steps):
        it0 = P.it_cnt
        gk.glp_simplex(P, parm)
        s = P.stats()
        piv += P.it_cnt - it0
        byts += s.bytes_pivots
        split["init"] += s.seconds_init
        split["eval"] += s.seconds_eval
        split["batches"] += s.seconds_batches
        split["reinvert"] += s.seconds_reinvert
        for k in ("reinversions", "refine_tries", "refinements", "refine_steps"):
            reinv[k] += getattr(s, k)
        reinv["refine_resid_max"] = max(reinv["refine_resid_max"], s.refine_resid_max)
    dt = time.perf_counter() - t0
    ctx.mark(2)
    adv["s_reinvert"] = round(adv["s_reinvert"], 3)
    print(json.dumps({"start": warm, "advance_seconds": round(t_adv, 2), "advance": adv, "pivots": piv, "seconds": round(dt, 4), "pivots_per_s": round(piv / dt, 1),
                      "bytes_per_pivot": round(byts / max(piv, 1)),
                      "GBps_algorithmic": round(byts / dt / 1e9, 1),
                      "ms_split": {k: round(1000 * v, 2) for k, v in split.items()},
                      "ms_per_reinversion": round(1000 * split["reinvert"] / max(reinv["reinversions"], 1), 2),
                      "newton_min_k": os.environ.get("GK_NEWTON_MIN_K", "default (512)"), **reinv}), flush=True)


if __name__ == "__main__":
    main()
