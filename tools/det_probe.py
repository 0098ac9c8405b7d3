#!/usr/bin/env python3
"""Determinism probe of the dual simplex on the dense generator: the same
solve REPS times in one process, every batch and re-inversion fingerprinted
by the engine (GK_DET_LOG, gk_engine.hip det_log), then the runs compared
line by line and the first divergent line printed.

usage: GK_DET_LOG=gpurun_out/det.log python tools/det_probe.py M N IT_LIM REPS [CALL_LIM [primal]]
       python tools/det_probe.py --compare gpurun_out/det.log [other.log]
CALL_LIM (default 0 = one call): it_lim of each glp_simplex call.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def runs_of(path):
    runs, cur = [], None
    for ln in open(path):
        if ln.startswith("=== run"):
            cur = []
            runs.append(cur)
        elif cur is not None:
            cur.append(ln.rstrip("\n"))
    return runs


def compare(runs):
    base = runs[0]
    out = []
    for r, other in enumerate(runs[1:], 1):
        first = None
        for i, (a, b) in enumerate(zip(base, other)):
            if a != b:
                first = i
                break
        if first is None and len(base) != len(other):
            first = min(len(base), len(other))
        if first is None:
            out.append(f"run {r}: identical to run 0 ({len(other)} lines)")
        else:
            out.append(f"run {r}: first divergence at line {first} of {len(base)}/{len(other)}")
            for j in range(max(0, first - 3), min(first + 2, len(base))):
                out.append("  0: " + base[j])
                if j < len(other):
                    out.append(f"  {r}: " + other[j])
    return out


def main():
    if sys.argv[1] == "--compare":
        runs = []
        for p in sys.argv[2:]:
            runs += runs_of(p)
        print("\n".join(compare(runs)))
        return
    import torch  # noqa: F401
    import __graft_entry__
    __graft_entry__.load_package()
    from glpk_js_amd import gk, problems
    m, n, it_lim, reps = (int(x) for x in sys.argv[1:5])
    call_lim = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    meth = gk.GLP_PRIMAL if len(sys.argv) > 6 and sys.argv[6] == "primal" else gk.GLP_DUAL
    log = os.environ.get("GK_DET_LOG")
    ctx = gk.Context(0)
    prob = problems.gen_dense(m, n, seed=42)
    for rep in range(reps):
        if log:
            with open(log, "a") as f:
                f.write(f"=== run {rep} pid {os.getpid()}\n")
        P = gk.GkProblem(ctx, prob)
        t0 = time.perf_counter()
        ret = 8
        while ret == 8 and P.it_cnt < it_lim:
            lim = min(call_lim or it_lim, it_lim - P.it_cnt)
            ret = gk.glp_simplex(P, gk.SMCP(meth=meth, it_lim=lim, msg_lev=gk.GLP_MSG_ERR))
        st = P.stats()
        print(json.dumps({"rep": rep, "ret": ret, "it_cnt": P.it_cnt, "obj": P.obj_val,
                          "seconds": round(time.perf_counter() - t0, 2), "reinversions": st.reinversions,
                          "refinements": st.refinements}), flush=True)
        del P
    if log:
        print("\n".join(compare(runs_of(log))), flush=True)


if __name__ == "__main__":
    main()
