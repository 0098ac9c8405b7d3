#!/usr/bin/env python3
"""Host timeline of the bench's glp_simplex calls (GK_CALL_LOG=1): C3 4096 x
16384, dual, it_lim 100 per call as bench.py's step; W warm-up calls, then K
calls whose "[gk call]" lines (label, microseconds from the call's entry)
show where the host time between the device's work goes; also the wall time
per call measured here.  usage: call_log.py [K] [W]"""
import os
import sys
import time

os.environ["GK_CALL_LOG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    prob = problems.gen_dense(4096, 16384, seed=42)
    ctx = gk.Context(0)
    P = gk.GkProblem(ctx, prob)
    P.touch_bounds()
    assert P.factorize() == 0
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR)
    for _ in range(W):
        gk.glp_simplex(P, parm)
    print("---- timed calls", file=sys.stderr, flush=True)
    for _ in range(K):
        t = time.perf_counter()
        ret = gk.glp_simplex(P, parm)
        dt = time.perf_counter() - t
        print(f"call ret {ret} it {P.it_cnt} wall {1e6 * dt:.0f} us", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
