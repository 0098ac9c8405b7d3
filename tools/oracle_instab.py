#!/usr/bin/env python3
"""The oracle (bit-exact C restatement of glpspx02.js) on C3 from the slack
basis in ONE glp_simplex(dual, it_lim) call: how many times its check_stab
fails ("numerical instability", glpspx02.js:1410 / message at :1668) on the
way, and at which iteration the last one happened.  Test infrastructure
(reads oracle/): run in the build container.

usage: python tools/oracle_instab.py [IT_LIM] [OUT.json]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
import orcpy  # noqa: E402
from glpk_js_amd import problems  # noqa: E402


def main():
    it_lim = int(sys.argv[1]) if len(sys.argv) > 1 else 64000
    out = sys.argv[2] if len(sys.argv) > 2 else None
    p = problems.gen_dense(4096, 16384, seed=42, keep_dense=False)
    o = orcpy.OracleProb(p)
    n0, _ = orcpy.instab_count()
    t0 = time.perf_counter()
    ret = o.simplex(meth=3, it_lim=it_lim)
    dt = time.perf_counter() - t0
    n1, last = orcpy.instab_count()
    r = o.result()
    res = {"instance": "C3 4096x16384 seed 42, dual, slack basis, one call", "it_lim": it_lim, "ret": ret,
           "it_cnt": r["it_cnt"], "obj_val": r["obj_val"], "seconds": round(dt, 1),
           "check_stab_failures": n1 - n0, "last_failure_it": last if n1 > n0 else None}
    print(json.dumps(res), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
