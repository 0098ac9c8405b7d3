"""glp_eval_tab_row (glpapi12.js:401) for batches of basic variables:
gk_bfd_eval_tab_rows against the reference's own rows.

tests/golden/tab_*.json (gen_golden.js, running the reference): a problem
(three of them scaled, so glp_btran's scaling is exercised), the basis
glp_simplex left, and glp_eval_tab_row's (ind, val) lists for up to 48
basic variables.

CPU: the restatement the device computes (rho = inv(B)' e_i of the unscaled
basis (I | -A) columns, alfa = rho' A_j for a non-basic structural, -rho_k
for a non-basic auxiliary) reproduces the reference's rows with numpy
(pins the formula and its sign conventions; parity to 1e-9 relative of the
row's largest entry).
GPU: the batch on the device — one MFMA GEMM on dense A, the per-row CSC
path otherwise or on request — matches the reference's rows to the same
tolerance, and the two device paths agree with each other."""
import os

import numpy as np
import pytest

from conftest import golden_files, load_golden
from glpk_js_amd import gk, problems

TAB = golden_files("tab_")
IDS = [os.path.basename(p)[4:-5] for p in TAB]
TOL = 1e-9


def ref_rows(d):
    m, n = d["m"], d["n"]
    out = np.zeros((len(d["tab_rows"]), m + n))
    for t, r in enumerate(d["tab_rows"]):
        out[t, np.asarray(r["ind"], dtype=np.int64) - 1] = r["val"]
    return out


def dense_A(d):
    A = np.zeros((d["m"], d["n"]))
    for j in range(d["n"]):
        lo, hi = d["A_ptr"][j], d["A_ptr"][j + 1]
        A[np.asarray(d["A_ind"][lo:hi]) - 1, j] = d["A_val"][lo:hi]
    return A


def close(ours, ref):
    scale = np.maximum(1.0, np.abs(ref).max(axis=1, initial=0.0))[:, None]
    return np.abs(ours - ref) <= TOL * scale


def test_fixtures_present():
    assert len(TAB) >= 5
    assert any(max(load_golden(p)["row_rii"]) != 1.0 or max(load_golden(p)["col_sjj"]) != 1.0 for p in TAB)


@pytest.mark.parametrize("path", TAB, ids=IDS)
def test_tab_rows_restatement_matches_reference(path):
    d = load_golden(path)
    m, n = d["m"], d["n"]
    A = dense_A(d)
    rs, cs = np.asarray(d["row_stat"]), np.asarray(d["col_stat"])
    basic = [k for k in range(1, m + n + 1) if (rs[k - 1] if k <= m else cs[k - m - 1]) == problems.GLP_BS]
    assert len(basic) == m
    B = np.zeros((m, m))
    for i, k in enumerate(basic):
        if k <= m:
            B[k - 1, i] = 1.0
        else:
            B[:, i] = -A[:, k - m - 1]
    ours = np.zeros((len(d["tab_rows"]), m + n))
    for t, r in enumerate(d["tab_rows"]):
        e = np.zeros(m)
        e[basic.index(r["k"])] = 1.0
        rho = np.linalg.solve(B.T, e)
        for k in range(1, m + 1):
            if rs[k - 1] != problems.GLP_BS:
                ours[t, k - 1] = -rho[k - 1]
        nb = cs != problems.GLP_BS
        ours[t, m:][nb] = (rho @ A)[nb]
    assert close(ours, ref_rows(d)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("path", TAB, ids=IDS)
def test_gpu_tab_rows_match_reference(gpu_ctx, path):
    d = load_golden(path)
    prob = problems.from_fixture(d)
    P = gk.GkProblem(gpu_ctx, prob)
    assert P.factorize() == 0
    ks = [r["k"] for r in d["tab_rows"]]
    ref = ref_rows(d)
    batch = P.eval_tab_rows(ks)
    per_row = P.eval_tab_rows(ks, per_row=True)
    assert close(batch, ref).all(), np.abs(batch - ref).max()
    assert close(per_row, ref).all(), np.abs(per_row - ref).max()
    assert close(batch, per_row).all()
    # the single-row API returns the reference's (ind, val) layout
    r0 = d["tab_rows"][0]
    ind, val = gk.glp_eval_tab_row(P, r0["k"])
    big = np.abs(ref[0]) > 1e-12 * max(1.0, np.abs(ref[0]).max())
    assert set(np.nonzero(big)[0] + 1) <= set(ind)


@pytest.mark.gpu
def test_gpu_tab_rows_errors(gpu_ctx):
    d = load_golden(TAB[0])
    P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
    assert P.factorize() == 0
    nonbasic = next(k for k in range(1, d["m"] + d["n"] + 1)
                    if (d["row_stat"][k - 1] if k <= d["m"] else d["col_stat"][k - d["m"] - 1]) != problems.GLP_BS)
    with pytest.raises(gk.GkError, match="must be basic"):
        P.eval_tab_rows([nonbasic])
    with pytest.raises(gk.GkError, match="out of range"):
        P.eval_tab_rows([d["m"] + d["n"] + 1])


@pytest.mark.gpu
def test_gpu_tab_rows_mfma_c3_block(gpu_ctx):
    """A 64-row batch on a dense 1024 x 4096 problem: the MFMA GEMM against
    the per-row path (and both against numpy on the factor's own rows)."""
    prob = problems.gen_dense(1024, 4096, seed=7)
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=300, msg_lev=gk.GLP_MSG_OFF)) in (0, problems.GLP_EITLIM)
    assert P.valid
    ks = [int(P.head[i]) for i in range(1, 65)]
    a = P.eval_tab_rows(ks)
    b = P.eval_tab_rows(ks, per_row=True)
    scale = np.maximum(1.0, np.abs(b).max(axis=1))[:, None]
    assert (np.abs(a - b) <= 1e-10 * scale).all()
