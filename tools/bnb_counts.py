#!/usr/bin/env python3
"""Node-LP and node counts of the batched search on every MIP fixture
(tests/golden/mip_*.json), solved as test_gpu_mip_matches_reference solves
them, beside the reference's counts.  The search is deterministic (DESIGN
§7), so these counts pin it: written to tests/golden/bnb_counts.json, which
the test compares exactly.

usage: python tools/bnb_counts.py [OUT]"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    out_p = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "bnb_counts.json")
    ctx = gk.Context(0)
    res = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "mip_*.json"))):
        d = json.load(open(path))
        prob = problems.from_fixture(d)
        P = gk.GkProblem(ctx, prob)
        assert gk.glp_simplex(P, gk.SMCP(**d["root"]["opts"])) == d["root"]["ret"]
        ret = gk.glp_intopt(P, gk.IOCP(msg_lev=gk.GLP_MSG_OFF))
        st = P.mip_stats
        name = os.path.basename(path)
        res[name] = {"ret": ret, "lp_solves": int(st.get("lp_solves", 0)), "nodes": int(st.get("nodes_created", 0)),
                     "reference_lp_solves": d["mip"].get("lp_solves")}
        print(name, res[name], file=sys.stderr, flush=True)
        del P
    json.dump({"note": "batched search counts on one MI355X (tools/bnb_counts.py); deterministic, compared "
                       "exactly by tests/test_gpu_mip.py", "counts": res}, open(out_p, "w"), indent=1)


if __name__ == "__main__":
    main()
