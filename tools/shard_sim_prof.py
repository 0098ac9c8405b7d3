#!/usr/bin/env python3
"""Column-sharded pricing, one rank's kernels as G ranks would run them
(DESIGN §8): C3 4096x16384 advanced to pivot START, then windows of STEPS
it_lim=100 dual calls with the pricing sharded over G = 1, then G simulated
ranks (GK_SHARD_ONE_RANK=1, GK_SHARD_SIM=G: one process forms every rank's
slice in turn, so under rocprofv3 each launch of the column pass and of
k_shard_aw is one rank's slice on an otherwise idle GPU).  Each window is
bracketed by gk_ctx_mark (tools/prof_stats.py --marked --window i).

usage: python tools/shard_sim_prof.py [G [START [STEPS]]]"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GK_SHARD_ONE_RANK"] = "1"
import torch  # noqa: F401,E402
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    start = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    ctx = gk.Context(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    comm = gk.Comm(ctx, 0, 1, f"127.0.0.1:{port}")
    P = gk.GkProblem(ctx, problems.gen_dense(4096, 16384, seed=42))
    adv = gk.SMCP(meth=gk.GLP_DUAL, it_lim=2000, msg_lev=gk.GLP_MSG_ERR)
    while P.it_cnt < start:
        assert gk.glp_simplex(P, adv) == 8
        print("advance", P.it_cnt, file=sys.stderr, flush=True)
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR)
    out = []
    for g in (1, G):
        os.environ["GK_SHARD_SIM"] = str(g)
        P.set_comm(comm)
        gk.glp_simplex(P, parm)                  # (buffers for this G, plan)
        torch.cuda.synchronize()
        ctx.mark(1)
        t0 = time.perf_counter()
        it0 = P.it_cnt
        for _ in range(steps):
            gk.glp_simplex(P, parm)
        dt = time.perf_counter() - t0
        ctx.mark(2)
        piv = P.it_cnt - it0
        out.append({"G": g, "pivots": piv, "seconds": round(dt, 4), "pivots_per_s": round(piv / dt, 1),
                    "exchanges": int(P.stats().shard_exchanges)})
        P.set_comm(None)
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"start": start, "steps": steps, "windows": out}))
    comm.close()


if __name__ == "__main__":
    main()
