#!/usr/bin/env python3
"""Secondary paths, one marked window each (for rocprofv3 --kernel-trace):
  0  C2s dual full solve           (surrogate of BASELINE configs[1])
  1  C2s primal full solve
  2  C3 4096x16384 primal, it_lim=300 from the slack basis
  3  dense 1024x4096 primal full solve
Prints one JSON line per case with the engine's host-side split."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (the library binds to torch's HIP runtime)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def run(ctx, tag, p, meth, it_lim=None):
    P = gk.GkProblem(ctx, p)
    kw = {"meth": meth, "msg_lev": gk.GLP_MSG_ERR}
    if it_lim:
        kw["it_lim"] = it_lim
    ctx.mark(1)
    t0 = time.perf_counter()
    ret = gk.glp_simplex(P, gk.SMCP(**kw))
    dt = time.perf_counter() - t0
    ctx.mark(2)
    s = P.stats()
    print(json.dumps({"case": tag, "ret": ret, "obj": P.obj_val, "pivots": P.it_cnt, "seconds": round(dt, 4),
                      "pivots_per_s": round(P.it_cnt / dt, 1), "reinversions": s.reinversions,
                      "batches": s.batches, "host_syncs": s.host_syncs,
                      "s_init": round(s.seconds_init, 4), "s_eval": round(s.seconds_eval, 4),
                      "s_batches": round(s.seconds_batches, 4), "s_reinvert": round(s.seconds_reinvert, 4),
                      "s_total": round(s.seconds_total, 4)}), flush=True)


def main():
    which = [int(a) for a in sys.argv[1:]] or [0, 1, 2, 3]
    ctx = gk.Context(0)
    for w in which:
        if w == 0:
            run(ctx, "c2s_dual", problems.gen_c2s(), gk.GLP_DUAL)
        elif w == 1:
            run(ctx, "c2s_primal", problems.gen_c2s(), gk.GLP_PRIMAL)
        elif w == 2:
            run(ctx, "c3_primal_300", problems.gen_dense(4096, 16384, seed=42), gk.GLP_PRIMAL, it_lim=300)
        elif w == 3:
            run(ctx, "d1024_primal", problems.gen_dense(1024, 4096, seed=42), gk.GLP_PRIMAL)


if __name__ == "__main__":
    main()
