#!/usr/bin/env python3
"""Oracle fixtures of large sparse LPs (the sparse factor path's parity at
sizes the oracle needs minutes to hours for): the oracle — the C restatement
of the reference's simplex, oracle/orcpy — solves the generated problem with
the dual simplex (meth = GLP_DUAL, as the GPU tests call it) and the result
goes to tests/golden/sparse_oracle_<name>.json.
usage: gen_sparse_oracle.py blocks K MB NB LINKS | c2s M N"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import problems  # noqa: E402
import orcpy  # noqa: E402


def main():
    kind, args = sys.argv[1], [int(x) for x in sys.argv[2:]]
    if kind == "blocks":
        K, mb, nb, links = args
        prob = problems.gen_blocks(K, mb, nb, links)
        name = f"blocks_{K}x{mb}x{nb}+{links}"
    else:
        m, n = args
        prob = problems.gen_c2s(m, n)
        name = f"c2s_{m}x{n}"
    o = orcpy.OracleProb(prob)
    t = time.time()
    ret = o.simplex(meth=3)
    res = o.result()
    out = {"problem": name, "kind": kind, "args": args, "m": prob.m, "n": prob.n, "nnz": int(len(prob.A_val)),
           "meth": "GLP_DUAL", "ret": ret, "obj": res["obj_val"], "it_cnt": res["it_cnt"],
           "oracle_seconds": round(time.time() - t, 1)}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"sparse_oracle_{name}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
