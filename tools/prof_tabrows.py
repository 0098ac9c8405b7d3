#!/usr/bin/env python3
"""Tableau rows on C3 (gk_bfd_eval_tab_rows, glp_eval_tab_row for a batch):
nk basic rows of the 4096 x 16384 problem after 300 dual pivots, by the MFMA
GEMM and by the per-row path, for rocprofv3 --kernel-trace --stats (the
kernel averages give TF/s = 2 nk m n / t).  usage: prof_tabrows.py [nk ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    nks = [int(a) for a in sys.argv[1:]] or [64, 128]
    m, n = 4096, 16384
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, problems.gen_dense(m, n, seed=42))
    assert P.factorize() == 0
    gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=300, msg_lev=gk.GLP_MSG_OFF))
    for nk in nks:
        ks = [int(P.head[i]) for i in range(1, nk + 1)]
        for per_row in (False, True):
            a = P.eval_tab_rows(ks, per_row=per_row)      # warm
            t0 = time.perf_counter()
            for _ in range(3):
                a = P.eval_tab_rows(ks, per_row=per_row)
            dt = (time.perf_counter() - t0) / 3
            print(f"nk={nk} {'per-row' if per_row else 'mfma   '}: {dt * 1e3:.2f} ms per call incl. copies, "
                  f"{2.0 * nk * m * n / dt / 1e12:.2f} TF/s call-level, |alfa|max {np.abs(a).max():.3g}", flush=True)


if __name__ == "__main__":
    main()
