#!/usr/bin/env python3
"""B&B timing split for one fixture (default C5s 12x30): wall time of
glp_intopt inside a gk_ctx_mark window (for rocprofv3 --kernel-trace), node
LP solves and batches."""
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
    name = sys.argv[1] if len(sys.argv) > 1 else "c5s_12x30"
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "mip_" + name + ".json")))
    ctx = gk.Context(0)
    for rep in range(3):
        P = gk.GkProblem(ctx, problems.from_fixture(d))
        assert gk.glp_simplex(P, gk.SMCP(msg_lev=gk.GLP_MSG_ERR)) == 0
        ctx.mark(1)
        t0 = time.perf_counter()
        ret = gk.glp_intopt(P, gk.IOCP(msg_lev=gk.GLP_MSG_ERR))
        dt = time.perf_counter() - t0
        ctx.mark(2)
        print(json.dumps({"rep": rep, "ret": ret, "obj": P.mip_obj, "seconds": round(dt, 4), **P.mip_stats}), flush=True)


if __name__ == "__main__":
    main()
