#!/usr/bin/env python3
"""A window of dual pivots on the sparse factor from a saved basis (the
m = 100,050 block-angular LP's late basis by default): pivots/s, the host LU
share and the sparse path's algorithmic bytes per pivot.

usage: python tools/sparse_window.py [--it N] [--basis F] [K [L]]
  K, L: problems.gen_blocks(K, 100, 200, L) (default 1000, 50);
  --basis F: row / column statuses saved by tools/sparse_big.py --save
  (default profiles/r04_blocks100k_basis_it644352.npz for K = 1000);
  --it N: pivots of the window (default 3000)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    it, basis = 3000, None
    args = sys.argv[1:]
    while args and args[0].startswith("--"):
        opt = args.pop(0)
        if opt == "--it":
            it = int(args.pop(0))
        elif opt == "--basis":
            basis = args.pop(0)
    K = int(args[0]) if args else 1000
    L = int(args[1]) if len(args) > 1 else 50
    if basis is None and K == 1000 and L == 50:
        basis = os.path.join(ROOT, "profiles", "r04_blocks100k_basis_it644352.npz")
    prob = problems.gen_blocks(K, 100, 200, L)
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, prob)
    if basis:
        z = np.load(basis)
        P.row_stat[1:prob.m + 1] = z["row_stat"]
        P.col_stat[1:prob.n + 1] = z["col_stat"]
        P.valid = 0
    ctx.mark(1)
    t0 = time.perf_counter()
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=it, msg_lev=gk.GLP_MSG_ERR))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.mark(2)
    st = P.stats()
    out = {"problem": prob.name, "m": prob.m, "n": prob.n, "basis": os.path.basename(basis) if basis else "slack",
           "ret": ret, "pivots": P.it_cnt, "seconds": round(dt, 3), "pivots_per_s": round(P.it_cnt / dt, 1),
           "factor_sparse": st.factor_sparse, "refactorizations": int(st.reinversions),
           "refactor_seconds": round(st.seconds_reinvert, 3), "host_lu_seconds": round(st.seconds_lu, 3),
           "host_lu_share": round(st.seconds_lu / dt, 4), "bytes_per_pivot": round(st.bytes_pivots / max(1, st.pivots)),
           # (the sparse pivot's algorithmic bytes, DESIGN §2f, over the window's wall time)
           "achieved_GBps": round(st.bytes_pivots / dt / 1e9, 1),
           "frac_of_hbm_peak": round(st.bytes_pivots / dt / 1e9 / 8000.0, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
