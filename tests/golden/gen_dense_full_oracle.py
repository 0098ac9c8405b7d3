#!/usr/bin/env python3
"""Full dual-simplex solves of the dense generator at
2048x8192 and 4096x16384 (C3) by the oracle — the bit-faithful C restatement
of glpspx02.js, pinned pivot-by-pivot against the reference (tests/golden/
lp_dense_*.json) — because the reference itself (Node, ~9 pivots/s at C3)
cannot finish them.  Writes tests/golden/dense_full_<m>x<n>.json with the
objective, statuses and iteration count.  Test infrastructure only.

usage: python tests/golden/gen_dense_full_oracle.py M N [SEED]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
import orcpy  # noqa: E402
from glpk_js_amd import problems  # noqa: E402


def main():
    m, n = int(sys.argv[1]), int(sys.argv[2])
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 42
    p = problems.gen_dense(m, n, seed=seed, keep_dense=False)
    o = orcpy.OracleProb(p)
    t0 = time.time()
    ret = o.simplex(meth=3)
    dt = time.time() - t0
    r = o.result()
    out = {"m": m, "n": n, "seed": seed, "meth": "dual", "ret": ret, "pbs_stat": r["pbs_stat"],
           "dbs_stat": r["dbs_stat"], "obj_val": r["obj_val"], "it_cnt": r["it_cnt"], "oracle_seconds": round(dt, 1)}
    path = os.path.join(ROOT, "tests", "golden", f"dense_full_{m}x{n}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
