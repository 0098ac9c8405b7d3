#!/usr/bin/env python3
"""Level structure of the sparse factor's four sweeps on a saved basis of the
block-angular LP (CPU only: gk_sp_selftest with GK_SP_LEVELS, which prints
steps/entries/long steps of every level of FTRAN L, FTRAN U, BTRAN U',
BTRAN L'), with a per-level trip model of the one-workgroup sweep.

usage: python tools/sp_levels.py [--basis F] [K [L]]"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    args = sys.argv[1:]
    basis = os.path.join(ROOT, "profiles", "r04_blocks100k_basis_it644352.npz")
    if args and args[0] == "--basis":
        basis = args[1]
        args = args[2:]
    if os.environ.get("GK_SP_LEVELS") is None:
        env = dict(os.environ, GK_SP_LEVELS="1", GK_SP_TIMES="1")
        r = subprocess.run([sys.executable, __file__, "--basis", basis] + args, env=env, capture_output=True, text=True)
        sys.stdout.write(r.stdout)
        names = ["FTRAN L", "FTRAN U", "BTRAN U'", "BTRAN L'"]
        lines = [ln for ln in r.stderr.splitlines() if ln.startswith("[gk sp levels]")]
        print("\n".join(ln for ln in r.stderr.splitlines() if ln.startswith("[gk sp times]") or ln.startswith("[gk sp plan]")))
        for name, ln in zip(names, lines[-4:]):
            body = ln.split("]", 1)[1].split("(")[0].split()
            lv = [tuple(int(x) for x in t.split("/")) for t in body]
            print(f"{name}: {len(lv)} levels, {sum(s for s, _, _ in lv)} steps, {sum(e for _, e, _ in lv)} entries")
            print("   " + " ".join(f"{s}/{e}/{g}" for s, e, g in lv))
        return
    import __graft_entry__
    __graft_entry__.load_package()
    from glpk_js_amd import gk, problems
    K = int(args[0]) if args else 1000
    Lk = int(args[1]) if len(args) > 1 else 50
    prob = problems.gen_blocks(K, 100, 200, Lk)
    z = np.load(basis)
    rs, cs = z["row_stat"], z["col_stat"]
    m = prob.m
    ptr, ind, val = [0, 1], [0], [0.0]
    for i in np.nonzero(rs == 1)[0]:
        ind.append(int(i) + 1)
        val.append(1.0)
        ptr.append(len(ind))
    for j in np.nonzero(cs == 1)[0]:
        lo, hi = prob.A_ptr[j], prob.A_ptr[j + 1]
        for t in range(lo, hi):
            ind.append(int(prob.A_ind[t]))
            val.append(-float(prob.A_val[t]))
        ptr.append(len(ind))
    assert len(ptr) == m + 2, (len(ptr), m)
    ptr, ind, val = (np.asarray(a, t) for a, t in ((ptr, np.int32), (ind, np.int32), (val, np.float64)))
    rng = np.random.default_rng(1)
    b, e, x, y, st = rng.standard_normal(m), rng.standard_normal(m), np.zeros(m), np.zeros(m), np.zeros(6, np.int64)
    f = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    L = gk.load_library()
    L.gk_sp_selftest.restype = C.c_int
    import time
    t0 = time.perf_counter()
    ret = L.gk_sp_selftest(m, f(ptr), f(ind), f(val), f(b), f(e), f(x), f(y), f(st))
    print(f"selftest (LU + solves build + plans + host sweeps) {1e3 * (time.perf_counter() - t0):.1f} ms")
    print("selftest ret", ret, "stats", st.tolist(), flush=True)
    # residuals of the two solves (the sweeps as the device runs them)
    import scipy.sparse as sps
    B = sps.csc_matrix((val[1:], ind[1:] - 1, ptr[1:] - 1), shape=(m, m))
    rx = np.abs(B @ x - b).max() / max(1.0, np.abs(x).max())
    ry = np.abs(B.T @ y - e).max() / max(1.0, np.abs(y).max())
    print(f"residual FTRAN {rx:.3e} BTRAN {ry:.3e}", flush=True)


if __name__ == "__main__":
    main()
