"""The sparse basis factor (glpk.js_amd/csrc/gk_sparse.hip), CPU side: the
Markowitz L U with threshold pivoting (the role of luf_factorize,
glpluf.js:1105) and the four level-scheduled sweeps of FTRAN / BTRAN (the
roles of luf_f_solve / luf_v_solve, glpluf.js:1227 / :1268), run on the host
in the order the device runs them (gk_sp_selftest), against numpy on bases of
(I | -A) drawn from the C2s generator and from block-angular LPs, plus
singular and permuted cases.  Tolerance: 1e-9 relative to the solution's
largest entry (the elimination order differs from numpy's LAPACK LU)."""
import ctypes as C
import os

import numpy as np
import pytest

from glpk_js_amd import gk, problems


def selftest(B):
    m = B.shape[0]
    L = gk.load_library()
    ptr, ind, val = [0, 1], [0], [0.0]
    for j in range(m):
        nz = np.nonzero(B[:, j])[0]
        for i in nz:
            ind.append(int(i) + 1)
            val.append(float(B[i, j]))
        ptr.append(len(ind))
    ptr = np.asarray(ptr, np.int32)
    ind = np.asarray(ind, np.int32)
    val = np.asarray(val, np.float64)
    rng = np.random.default_rng(m)
    b = rng.standard_normal(m)
    e = rng.standard_normal(m)
    x = np.zeros(m)
    y = np.zeros(m)
    st = np.zeros(6, np.int64)
    f = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    L.gk_sp_selftest.restype = C.c_int
    ret = L.gk_sp_selftest(m, f(ptr), f(ind), f(val), f(b), f(e), f(x), f(y), f(st))
    return ret, b, e, x, y, st


def basis_from(prob, head):
    """columns of (I | -A) for the variables in head (1-based)"""
    m = prob.m
    A = np.zeros((m, prob.n))
    for j in range(prob.n):
        lo, hi = prob.A_ptr[j], prob.A_ptr[j + 1]
        A[prob.A_ind[lo:hi] - 1, j] = prob.A_val[lo:hi]
    cols = []
    for k in head:
        cols.append(np.eye(m)[:, k - 1] if k <= m else -A[:, k - m - 1])
    return np.stack(cols, axis=1)


def check(B):
    ret, b, e, x, y, st = selftest(B)
    assert ret == 0
    xr = np.linalg.solve(B, b)
    yr = np.linalg.solve(B.T, e)
    assert np.abs(x - xr).max() <= 1e-9 * max(1.0, np.abs(xr).max()), np.abs(x - xr).max()
    assert np.abs(y - yr).max() <= 1e-9 * max(1.0, np.abs(yr).max()), np.abs(y - yr).max()
    return st


@pytest.mark.parametrize("m,n,nstruct", [(60, 120, 30), (200, 400, 120), (400, 800, 400)])
def test_sparse_factor_c2s_bases(m, n, nstruct):
    prob = problems.gen_c2s(m, n, seed=7)
    rng = np.random.default_rng(m)
    for _ in range(5):
        # a random mixed basis: nstruct structural columns, slacks for the rest
        for _try in range(50):
            cols = rng.choice(n, nstruct, replace=False) + m + 1
            B = basis_from(prob, list(cols))
            A = B[:, :nstruct]
            # complete by slacks of rows that keep B nonsingular
            q, r, piv = __import__("scipy.linalg", fromlist=["qr"]).qr(A.T, pivoting=True)
            rank = int((np.abs(np.diag(r)) > 1e-9 * np.abs(r).max()).sum()) if nstruct else 0
            if rank == nstruct:
                break
        used = set(piv[:nstruct].tolist()) if nstruct else set()
        rows = [i for i in range(m) if i not in used]
        head = list(cols) + [i + 1 for i in rows]
        B = basis_from(prob, head)
        if abs(np.linalg.slogdet(B)[0]) == 0:
            continue
        st = check(B)
        assert st[1] >= m and st[2] >= 1


def test_sparse_factor_permuted_triangular():
    # a permuted upper-triangular matrix: no fill, levels = the dependency depth
    m = 50
    rng = np.random.default_rng(3)
    U = np.triu(rng.uniform(0.5, 1.5, (m, m)) * (rng.random((m, m)) < 0.1)) + np.eye(m) * 2
    P = np.eye(m)[rng.permutation(m)]
    Q = np.eye(m)[rng.permutation(m)]
    st = check(P @ U @ Q)
    assert st[0] == 0                        # triangular: no L multipliers


def test_sparse_factor_dense_block():
    m = 40
    rng = np.random.default_rng(5)
    B = rng.uniform(-1, 1, (m, m)) + np.eye(m) * 0.1
    st = check(B)
    assert st[0] + st[1] <= m * m + m


def test_sparse_factor_singular():
    m = 30
    rng = np.random.default_rng(9)
    B = rng.uniform(0.5, 1.5, (m, m)) * (rng.random((m, m)) < 0.2) + np.eye(m)
    B[:, 7] = B[:, 3] * 2.0
    ret, *_ = selftest(B)
    assert ret == 1


def test_sparse_factor_block_angular():
    # blocks of C2s-like columns plus linking rows (the m = 100,000 test's structure)
    rng = np.random.default_rng(11)
    K, mb, L = 6, 20, 3
    m = K * mb + L
    cols = []
    for k in range(K):
        for _ in range(mb // 2):
            c = np.zeros(m)
            c[k * mb + rng.choice(mb, 4, replace=False)] = rng.uniform(0.5, 1.5, 4)
            c[K * mb + rng.integers(L)] = rng.uniform(0.5, 1.5)
            cols.append(-c)
    B = np.stack(cols, axis=1)
    nst = B.shape[1]
    q, r, piv = __import__("scipy.linalg", fromlist=["qr"]).qr(B.T, pivoting=True)
    used = set(piv[:nst].tolist())
    rows = [i for i in range(m) if i not in used]
    B = np.concatenate([B, np.eye(m)[:, rows]], axis=1)
    check(B)


def test_sparse_oracle_fixtures_regenerate_their_problems():
    """The large sparse oracle fixtures (tests/golden/sparse_oracle_*.json,
    written by gen_sparse_oracle.py) name problems the generators still
    produce: the same size and number of nonzeros, and a finite objective."""
    import glob
    import json
    import math
    from glpk_js_amd import problems
    paths = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "sparse_oracle_*.json")))
    assert paths
    for p in paths:
        d = json.load(open(p))
        prob = problems.gen_blocks(*d["args"]) if d["kind"] == "blocks" else problems.gen_c2s(*d["args"])
        assert (prob.m, prob.n, len(prob.A_val)) == (d["m"], d["n"], d["nnz"]), p
        assert d["ret"] == 0 and math.isfinite(d["obj"])
