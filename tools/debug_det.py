# determinism probe: the same B&B three times in one process
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import __graft_entry__
__graft_entry__.load_package()
from glpk_js_amd import gk, problems
ctx = gk.Context(0)
for name in sys.argv[1:]:
    d = json.load(open(os.path.join(ROOT, "tests", "golden", f"mip_{name}.json")))
    for rep in range(5):
        P = gk.GkProblem(ctx, problems.from_fixture(d))
        gk.glp_simplex(P, gk.SMCP(**d["root"]["opts"]))
        ret = gk.glp_intopt(P, gk.IOCP(msg_lev=gk.GLP_MSG_OFF))
        print(name, rep, ret, P.mip_obj, P.mip_stats, flush=True)
