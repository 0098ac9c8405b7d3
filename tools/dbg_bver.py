#!/usr/bin/env python3
"""test_gpu_bounds_version_fast_init_bit_identical's two chains, the first
difference printed (debugging aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402

ctx = gk.Context(0)
outs = []
for declared in (False, True):
    prob = problems.gen_dense(256, 1024, seed=3)
    P = gk.GkProblem(ctx, prob)
    if declared:
        P.touch_bounds()
    trace = []
    for k in range(12):
        if k == 6:
            P.row_ub[5] *= 0.5
            if declared:
                P.touch_bounds()
        ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=40, msg_lev=gk.GLP_MSG_OFF))
        st = P.stats()
        trace.append((ret, P.it_cnt, P.obj_val.hex(), bytes(P.row_stat), bytes(P.col_stat), int(st.resident),
                      int(st.evals_skipped), int(st.reinversions)))
    outs.append(trace)
for k, (a, b) in enumerate(zip(*outs)):
    same = a[:5] == b[:5]
    print(k, "same" if same else "DIFF", a[0], a[1], a[2], b[2], "resident", a[5], b[5], "skipped", a[6], b[6],
          "reinv", a[7], b[7], "rowstat diffs", sum(x != y for x, y in zip(a[3], b[3])),
          "colstat diffs", sum(x != y for x, y in zip(a[4], b[4])), flush=True)
