"""B&B wall time of the bench's MIP configs (gap, C5s 12x30) with the device
node records on and off (GK_BNB_WARM is read per search)
(set GK_BNB_LOG=1 for the driver's own time split on stderr; its
time stamps cost ~0.1 us a node, so time without it).  Usage:
    python tools/bnb_time.py [--log=N] [--hostprof=US] [reps] [names...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
for a in list(sys.argv[1:]):
    if a.startswith("--log="):                  # GK_BNB_LOG level (read once per process)
        os.environ["GK_BNB_LOG"] = a[6:]
        sys.argv.remove(a)
    elif a.startswith("--hostprof="):           # GK_HOST_PROF sampling interval (us)
        os.environ["GK_HOST_PROF"] = a[11:]
        sys.argv.remove(a)

import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    names = sys.argv[2:] or ["gap", "c5s_12x30"]
    ctx = gk.Context(0)
    for name in names:
        d = json.load(open(os.path.join(ROOT, "tests", "golden", f"mip_{name}.json")))
        prob = problems.from_fixture(d)
        for warm in ("1", "0"):
            os.environ["GK_BNB_WARM"] = warm
            for r in range(reps + 1):          # the first search is a warm-up
                P = gk.GkProblem(ctx, prob.copy())
                assert gk.glp_simplex(P, gk.SMCP(msg_lev=gk.GLP_MSG_ERR)) == 0
                sys.stderr.flush()
                t0 = time.perf_counter()
                ret = gk.glp_intopt(P, gk.IOCP(msg_lev=gk.GLP_MSG_ERR))
                dt = time.perf_counter() - t0
                print(json.dumps({"name": name, "records": warm == "1", "rep": r - 1, "ret": ret,
                                  "obj": P.mip_obj, "ref_obj": d["mip"]["mip_obj"], "seconds": round(dt, 4),
                                  **P.mip_stats}), flush=True)
                assert abs(P.mip_obj - d["mip"]["mip_obj"]) <= 1e-9 * max(1.0, abs(d["mip"]["mip_obj"]))


if __name__ == "__main__":
    main()
