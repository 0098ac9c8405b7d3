"""KKT certificate of an optimal basic solution of the dense generator's LP
(maximize c'x, A x <= b, x >= 0) — a size-independent
parity property for full-size solves the reference cannot finish (its Node
path runs ~9 pivots/s at C3).  Primal feasibility, dual feasibility of the
reported row duals y and reduced costs d = c - A'y, complementary slackness
and a zero duality gap c'x = b'y together prove the objective optimal."""
import numpy as np


def dense_kkt(P, prob, tol=1e-7):
    """Returns a dict of the residuals; raises AssertionError on a violation.
    P: a solved GkProblem; prob: its Problem with the dense matrix kept."""
    A = prob.dense                        # m x n, unscaled
    b = prob.row_ub
    c = prob.col_coef
    x = P.col_prim[1:]
    y = P.row_dual[1:]
    d = P.col_dual[1:]
    ax = A @ x
    scale_b = 1.0 + np.abs(b).max()
    res = {
        "primal_bound": float(max(0.0, -x.min())),
        "primal_rows": float(max(0.0, (ax - b).max()) / scale_b),
        "row_act": float(np.abs(ax - P.row_prim[1:]).max() / scale_b),
        # maximisation: y >= 0 on <= rows, reduced costs <= 0 on x >= 0
        "dual_rows": float(max(0.0, -y.min())),
        "dual_cols": float(max(0.0, (c - A.T @ y).max()) / (1.0 + np.abs(c).max())),
        "reduced_costs": float(np.abs((c - A.T @ y) - d).max() / (1.0 + np.abs(c).max())),
        "compl_cols": float(np.abs(d * x).max() / (1.0 + np.abs(c @ x))),
        "compl_rows": float(np.abs(y * (b - ax)).max() / (1.0 + np.abs(c @ x))),
    }
    pobj, dobj = float(c @ x), float(b @ y)
    res["gap"] = abs(pobj - dobj) / max(1.0, abs(pobj))
    res["obj_vs_reported"] = abs(pobj + prob.c0 - P.obj_val) / max(1.0, abs(pobj))
    for k, v in res.items():
        assert v <= (1e-9 if k in ("gap", "obj_vs_reported") else tol), (k, v, res)
    return res


def sparse_kkt(P, prob, tol=1e-7):
    """The certificate of dense_kkt for a sparse problem of the generators'
    form (maximize c'x, A x <= b, x >= 0; A in the Problem's CSC arrays)."""
    import scipy.sparse as sp
    cols = np.repeat(np.arange(prob.n), np.diff(prob.A_ptr))
    A = sp.csc_matrix((prob.A_val, (prob.A_ind - 1, cols)), shape=(prob.m, prob.n))
    b, c = prob.row_ub, prob.col_coef
    x, y, d = P.col_prim[1:], P.row_dual[1:], P.col_dual[1:]
    ax = A @ x
    aty = A.T @ y
    scale_b = 1.0 + np.abs(b).max()
    res = {
        "primal_bound": float(max(0.0, -x.min())),
        "primal_rows": float(max(0.0, (ax - b).max()) / scale_b),
        "row_act": float(np.abs(ax - P.row_prim[1:]).max() / scale_b),
        "dual_rows": float(max(0.0, -y.min())),
        "dual_cols": float(max(0.0, (c - aty).max()) / (1.0 + np.abs(c).max())),
        "reduced_costs": float(np.abs((c - aty) - d).max() / (1.0 + np.abs(c).max())),
        "compl_cols": float(np.abs(d * x).max() / (1.0 + np.abs(c @ x))),
        "compl_rows": float(np.abs(y * (b - ax)).max() / (1.0 + np.abs(c @ x))),
    }
    pobj, dobj = float(c @ x), float(b @ y)
    res["gap"] = abs(pobj - dobj) / max(1.0, abs(pobj))
    res["obj_vs_reported"] = abs(pobj + prob.c0 - P.obj_val) / max(1.0, abs(pobj))
    for k, v in res.items():
        assert v <= (1e-9 if k in ("gap", "obj_vs_reported") else tol), (k, v, res)
    return res
