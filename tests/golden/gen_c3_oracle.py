#!/usr/bin/env python3
"""C3 (4096 x 16384, seed 42) at full size through the oracle — the
bit-faithful C restatement of glpspx02.js, itself pinned pivot by pivot on the
reference's C3 run (tests/golden/c3_itlim.json.gz, gen_golden.js --c3) —
along the bench's call sequence: glp_simplex(SMCP{meth: GLP_DUAL, it_lim:
100}) repeated from the slack basis, each call continuing from the basis the
previous one left.  The reference (Node, ~9 pivots/s here) would take hours
for this window; the oracle takes about a minute.

Writes tests/golden/c3_oracle_window.json.gz: after calls 3 (pivot 300) and
25 (pivot 2500, the end of the bench's warm-up + timed window) the return
code, statuses, objective, primal and dual values, the pivot trace of all
calls, and the number of "numerical instability" restarts the restatement
went through (check_stab, glpspx02.js:1666-1678).  Test infrastructure only.

usage: python tests/golden/gen_c3_oracle.py [CALLS]"""
import gzip
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

KEEP = (3, 25)


def snap(o, ret, trace, k, dt):
    r = o.result()
    return {"call": k, "ret": ret, "it_cnt": r["it_cnt"], "pbs_stat": r["pbs_stat"], "dbs_stat": r["dbs_stat"],
            "obj_val": r["obj_val"], "row_stat": r["row_stat"].tolist(), "col_stat": r["col_stat"].tolist(),
            "row_prim": r["row_prim"].tolist(), "col_prim": r["col_prim"].tolist(),
            "row_dual": r["row_dual"].tolist(), "col_dual": r["col_dual"].tolist(),
            "trace": [list(t) for t in trace], "instab": orcpy.instab_count()[0], "seconds": round(dt, 1)}


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else max(KEEP)
    p = problems.gen_dense(4096, 16384, seed=42, keep_dense=False)
    o = orcpy.OracleProb(p)
    trace, out, rets = [], [], []
    t0 = time.time()
    for k in range(1, calls + 1):
        ret = o.simplex(trace=trace, meth=3, it_lim=100)
        rets.append(ret)
        n_in, it_in = orcpy.instab_count()
        print(f"call {k}: ret {ret} it_cnt {o.result()['it_cnt']} instab {n_in} (last at {it_in}) "
              f"{time.time() - t0:.1f}s", flush=True)
        if k in KEEP:
            out.append(snap(o, ret, trace, k, time.time() - t0))
    d = {"name": "c3_oracle_window", "gen": {"kind": "dense", "m": 4096, "n": 16384, "seed": 42},
         "opts": {"meth": 3, "it_lim": 100}, "rets": rets, "states": out}
    path = os.path.join(ROOT, "tests", "golden", "c3_oracle_window.json.gz")
    with gzip.open(path, "wt") as f:
        json.dump(d, f)
    print("wrote", path)


if __name__ == "__main__":
    main()
