"""Chains of it_lim=100 dual calls to the optimum with the end-of-call
epilogue on and off (GK_EPILOGUE): calls, return code, objective, and the
first call whose state differs."""
import os
import sys
sys.path.insert(0, os.getcwd())
import __graft_entry__
__graft_entry__.load_package()
from glpk_js_amd import gk, problems
ctx = gk.Context(0)
for (m, n, seed) in ((1024, 4096, 42), (512, 2048, 7)):
    prob = problems.gen_dense(m, n, seed=seed)
    res = {}
    for on in ("1", "0"):
        os.environ["GK_EPILOGUE"] = on
        P = gk.GkProblem(ctx, prob)
        out = []
        for k in range(600):
            ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR))
            out.append((ret, P.it_cnt, float(P.obj_val).hex(), P.col_prim[1:].tobytes(), P.row_dual[1:].tobytes()))
            if ret != 8:
                break
        res[on] = out
        print(m, n, "epilogue", on, "calls", len(out), "ret", ret, "it", P.it_cnt, "obj", P.obj_val, flush=True)
    diff = [k for k, (a, b) in enumerate(zip(res["1"], res["0"])) if a != b]
    print("first differing call", diff[:1], flush=True)
