#!/usr/bin/env python3
"""Large sparse LPs through the sparse factor path (gk_sparse.hip) on one
GPU: the block-angular generator (problems.gen_blocks) or C2s, whole dual
solve, progress lines every out_frq pivots (stderr), then one JSON line with
pivots/s, refactorization time, the factor's size and a KKT certificate.
Usage: sparse_big.py [--sparse] blocks K [links [mb nb]] | c2s M N
(--sparse: GK_SPARSE=1, the sparse factor also below m = 65536)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402
from kkt import sparse_kkt  # noqa: E402


def main():
    if sys.argv[1] == "--sparse":
        os.environ["GK_SPARSE"] = "1"
        del sys.argv[1]
    os.environ.setdefault("GK_SPARSE_LOG", "1")
    kind = sys.argv[1]
    t0 = time.time()
    if kind == "blocks":
        K = int(sys.argv[2])
        L = int(sys.argv[3]) if len(sys.argv) > 3 else max(5, K // 20)
        mb = int(sys.argv[4]) if len(sys.argv) > 4 else 100
        nb = int(sys.argv[5]) if len(sys.argv) > 5 else 200
        prob = problems.gen_blocks(K, mb, nb, L)
    else:
        prob = problems.gen_c2s(int(sys.argv[2]), int(sys.argv[3]))
    t_gen = time.time() - t0
    print(f"[sparse_big] {prob.name}: m={prob.m} n={prob.n} nnz={len(prob.A_val)} generated in {t_gen:.1f}s",
          file=sys.stderr, flush=True)
    gk.glp_set_print_func(lambda s: print(s, file=sys.stderr, flush=True))
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, prob)
    t1 = time.time()
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ON, out_frq=2000))
    dt = time.time() - t1
    st = P.stats()
    out = {"problem": prob.name, "m": prob.m, "n": prob.n, "nnz": int(len(prob.A_val)), "ret": ret,
           "obj": P.obj_val, "pivots": P.it_cnt, "seconds": round(dt, 2), "pivots_per_s": round(P.it_cnt / dt, 1),
           "refactorizations": int(st.reinversions), "refactor_seconds": round(st.seconds_reinvert, 2),
           "sparse_env": os.environ.get("GK_SPARSE")}
    try:
        res = sparse_kkt(P, prob)
        out["kkt"] = {"certified": True, "gap": res["gap"], "max_residual": max(res.values())}
    except AssertionError as e:
        out["kkt"] = {"certified": False, "violation": str(e)[:300]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
