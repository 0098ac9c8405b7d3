#!/usr/bin/env python3
"""Large sparse LPs through the sparse factor path (gk_sparse.hip) on one
GPU: the block-angular generator (problems.gen_blocks) or C2s, whole dual
solve, progress lines every out_frq pivots (stderr), then one JSON line with
pivots/s, refactorization time, the factor's size and a KKT certificate.
Usage: sparse_big.py [--sparse] [--tm SECS] [--save F] [--load F] [--wide N] blocks K [links [mb nb]] | c2s M N
(--sparse: GK_SPARSE=1, the sparse factor also below m = 65536; --tm: the
call's tm_lim in seconds (GLP_ETMLIM at the limit); --save F: the final
row / column statuses into F (.npz); --load F: start from the statuses in F,
as glp_set_row_stat / glp_set_col_stat would set them — a solve longer than
one GPU session runs as a chain of tm_lim calls, each warm-started from the
basis the previous one saved; --wide N: GK_SP_WIDE, the level-0 size from
which a sweep's first level runs on the whole grid)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402
from kkt import sparse_kkt  # noqa: E402


def main():
    tm, save, load = None, None, None
    while sys.argv[1].startswith("--"):
        opt = sys.argv.pop(1)
        if opt == "--sparse":
            os.environ["GK_SPARSE"] = "1"
        elif opt == "--tm":
            tm = int(sys.argv.pop(1))
        elif opt == "--save":
            save = sys.argv.pop(1)
        elif opt == "--load":
            load = sys.argv.pop(1)
        elif opt == "--wide":
            os.environ["GK_SP_WIDE"] = sys.argv.pop(1)
        else:
            raise SystemExit(f"unknown option {opt}")
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
    t_beg = time.time()
    gk.glp_set_print_func(lambda s: print(f"[{time.time() - t_beg:8.1f}s] {s}", file=sys.stderr, flush=True))
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, prob)
    if load:
        z = np.load(load)
        assert z["row_stat"].shape == (prob.m,) and z["col_stat"].shape == (prob.n,)
        P.row_stat[1:prob.m + 1] = z["row_stat"]
        P.col_stat[1:prob.n + 1] = z["col_stat"]
        P.valid = 0
        print(f"[sparse_big] warm start from {load} ({int(z['pivots'])} pivots before)", file=sys.stderr, flush=True)
    smcp = gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ON, out_frq=2000)
    if tm:
        smcp.tm_lim = 1000 * tm
    t1 = time.time()
    ret = gk.glp_simplex(P, smcp)
    dt = time.time() - t1
    if save:
        before = int(np.load(load)["pivots"]) if load else 0
        np.savez_compressed(save, row_stat=np.asarray(P.row_stat[1:prob.m + 1], np.int8),
                            col_stat=np.asarray(P.col_stat[1:prob.n + 1], np.int8), pivots=before + P.it_cnt)
    st = P.stats()
    out = {"problem": prob.name, "m": prob.m, "n": prob.n, "nnz": int(len(prob.A_val)), "ret": ret,
           "obj": P.obj_val, "pivots": P.it_cnt, "seconds": round(dt, 2), "pivots_per_s": round(P.it_cnt / dt, 1),
           "refactorizations": int(st.reinversions), "refactor_seconds": round(st.seconds_reinvert, 2),
           "sparse_env": os.environ.get("GK_SPARSE"), "warm_start": load,
           "pivots_before": int(np.load(load)["pivots"]) if load else 0}
    try:
        res = sparse_kkt(P, prob)
        out["kkt"] = {"certified": True, "gap": res["gap"], "max_residual": max(res.values())}
    except AssertionError as e:
        out["kkt"] = {"certified": False, "violation": str(e)[:300]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
