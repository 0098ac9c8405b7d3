"""The sparse factor path on the GPU (gk_sparse.hip: B0 = L U, level-
scheduled sweeps, Schur-complement updates), forced onto
problems the explicit inverse would serve (GK_SPARSE=1) and taken by itself
beyond its limit (m > 65535).

Bar (north star): the reference's return code and statuses, objective
within 1e-9 relative (tests/golden lp_* dual runs, pinned by the reference
itself; the block-angular generator pinned by the oracle — the bit-faithful
C restatement of the reference's dual simplex — run in the test), and a KKT
certificate of every optimum (tests/kkt.py).  The pivot path is not
compared: the factor rounds differently from the reference's FT-LU."""
import os
import sys

import numpy as np
import pytest

from conftest import golden_files, load_golden
from glpk_js_amd import gk, problems
from kkt import sparse_kkt
from test_gpu_lp import check_solution

pytestmark = pytest.mark.gpu

SPARSE_RUNS = []
for path in golden_files("lp_"):
    d = load_golden(path)
    if d.get("gen", {}).get("kind") == "dense":
        continue
    for r, run in enumerate(d["runs"]):
        if not run["opts"].get("it_lim"):
            SPARSE_RUNS.append(pytest.param(path, r, id=f"{os.path.basename(path)[3:-5]}-{r}-m{run['opts'].get('meth', 1)}"))


@pytest.fixture
def sparse_on(monkeypatch):
    monkeypatch.setenv("GK_SPARSE", "1")


@pytest.mark.parametrize("path,run_index", SPARSE_RUNS)
def test_gpu_sparse_matches_reference(gpu_ctx, sparse_on, path, run_index):
    """Every LP fixture with sparse A, both methods (primal, dual, dual-then-
    primal), on the sparse factor."""
    d = load_golden(path)
    run = d["runs"][run_index]
    prob = problems.from_fixture(d)
    P = gk.GkProblem(gpu_ctx, prob)
    ret = gk.glp_simplex(P, gk.SMCP(**run["opts"]))
    assert ret == run["ret"]
    assert (P.pbs_stat, P.dbs_stat) == (run["pbs_stat"], run["dbs_stat"])
    if P.pbs_stat == problems.GLP_FEAS and P.dbs_stat == problems.GLP_FEAS:
        ref = run["obj_val"]
        assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
        check_solution(P)


def test_gpu_sparse_c2s_full_dual(gpu_ctx, sparse_on):
    """C2s 821 x 1571 (the configs[1] surrogate), whole dual solve on the
    sparse factor: the reference's objective 357.82820943518834 (SURVEY.md
    §4), KKT-certified."""
    prob = problems.gen_c2s()
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    assert abs(P.obj_val - 357.82820943518834) <= 1e-9 * 357.82820943518834, P.obj_val
    sparse_kkt(P, prob)
    st = P.stats()
    print("c2s sparse:", P.it_cnt, "pivots", st.reinversions, "refactorizations", st.seconds_total, "s")


@pytest.mark.parametrize("blocks,links", [(10, 5), (40, 10)])
def test_gpu_sparse_blocks_match_oracle(gpu_ctx, sparse_on, oracle, blocks, links):
    """Block-angular LPs (problems.gen_blocks, 100 x 200 blocks + linking
    rows): the oracle's objective (≤ 1e-9), KKT-certified."""
    prob = problems.gen_blocks(blocks, 100, 200, links)
    o = oracle.OracleProb(prob)
    assert o.simplex(meth=3) == 0
    ref = o.result()["obj_val"]
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    assert (P.pbs_stat, P.dbs_stat) == (problems.GLP_FEAS, problems.GLP_FEAS)
    assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
    sparse_kkt(P, prob)
    st = P.stats()
    print(f"blocks {blocks}: {P.it_cnt} pivots, {st.reinversions} refactorizations, {st.seconds_total:.2f} s "
          f"({P.it_cnt / st.seconds_total:.0f} pivots/s), refactor {st.seconds_reinvert:.2f} s")


SPARSE_FIXTURES = [pytest.param(p, id=os.path.basename(p)[len("sparse_oracle_"):-5])
                   for p in golden_files("sparse_oracle_")]


@pytest.mark.parametrize("path", SPARSE_FIXTURES)
def test_gpu_sparse_large_matches_oracle_fixture(gpu_ctx, sparse_on, path):
    """Sparse LPs the oracle needs minutes to hours for, solved once in the
    build container by tests/golden/gen_sparse_oracle.py (the C restatement
    of the reference's dual simplex): return code and objective (≤ 1e-9) of
    the fixture, KKT-certified.  blocks_200x100x200+20 (m = 20,020, n =
    40,000): the oracle took 89,265 iterations in 275 s."""
    d = load_golden(path)
    prob = (problems.gen_blocks(*d["args"]) if d["kind"] == "blocks" else problems.gen_c2s(*d["args"]))
    assert (prob.m, prob.n, len(prob.A_val)) == (d["m"], d["n"], d["nnz"])
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == d["ret"]
    assert abs(P.obj_val - d["obj"]) <= 1e-9 * max(1.0, abs(d["obj"])), (P.obj_val, d["obj"])
    sparse_kkt(P, prob)
    st = P.stats()
    print(f"{d['problem']}: {P.it_cnt} pivots (oracle {d['it_cnt']}), {st.seconds_total:.1f} s")


def test_gpu_sparse_c2s_full_primal(gpu_ctx, sparse_on):
    """C2s, whole primal solve on the sparse factor: the reference's primal
    objective 357.82820943518863, KKT-certified."""
    prob = problems.gen_c2s()
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_PRIMAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    assert abs(P.obj_val - 357.82820943518863) <= 1e-9 * 357.82820943518863, P.obj_val
    sparse_kkt(P, prob)


@pytest.mark.parametrize("blocks,links", [(10, 5), (40, 10)])
def test_gpu_sparse_blocks_primal_match_oracle(gpu_ctx, sparse_on, oracle, blocks, links):
    prob = problems.gen_blocks(blocks, 100, 200, links)
    o = oracle.OracleProb(prob)
    assert o.simplex(meth=1) == 0
    ref = o.result()["obj_val"]
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_PRIMAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
    sparse_kkt(P, prob)


def test_gpu_sparse_beyond_explicit_limit(gpu_ctx):
    """m > 65535 takes the sparse factor by itself (no GK_SPARSE): a block-
    angular LP of 65,650 rows, the first 2,000 pivots of each method through
    it (it_lim), statuses and bounds kept (the whole solves are
    tools/sparse_big.py runs, profiles/r04_sparse_*)."""
    prob = problems.gen_blocks(656, 100, 200, 50)
    assert prob.m > 65535
    for meth in (gk.GLP_DUAL, gk.GLP_PRIMAL):
        P = gk.GkProblem(gpu_ctx, prob.copy())
        ret = gk.glp_simplex(P, gk.SMCP(meth=meth, it_lim=2000, msg_lev=gk.GLP_MSG_ERR))
        assert ret == problems.GLP_EITLIM and P.it_cnt == 2000
        check_solution(P)


def test_gpu_sparse_phase_and_limits(gpu_ctx, sparse_on):
    """it_lim stops and continuation on the sparse factor: a chain of short
    calls reaches the same optimum as one call (the factor, its Schur chain
    and the resident working set carried across calls)."""
    prob = problems.gen_blocks(10, 100, 200, 5)
    P = gk.GkProblem(gpu_ctx, prob)
    while True:
        ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=250, msg_lev=gk.GLP_MSG_ERR))
        assert ret in (0, problems.GLP_EITLIM)
        if ret == 0:
            break
    Q = gk.GkProblem(gpu_ctx, prob.copy())
    assert gk.glp_simplex(Q, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    assert abs(P.obj_val - Q.obj_val) <= 1e-9 * abs(Q.obj_val)
    sparse_kkt(P, prob)


def test_gpu_sparse_warm_start_from_statuses(gpu_ctx, sparse_on):
    """A solve continued from saved row / column statuses (glp_set_row_stat /
    glp_set_col_stat, then glp_simplex: glp_factorize of the advanced basis
    through the sparse factor, gk_bfd_factorize_csc) reaches the optimum of
    one uninterrupted solve; the factor glp_factorize leaves serves FTRAN /
    BTRAN (glp_ftran / glp_btran) against numpy."""
    prob = problems.gen_blocks(10, 100, 200, 5)
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=1500, msg_lev=gk.GLP_MSG_ERR)) == problems.GLP_EITLIM
    Q = gk.GkProblem(gpu_ctx, prob.copy())
    Q.row_stat[1:prob.m + 1] = P.row_stat[1:prob.m + 1]
    Q.col_stat[1:prob.n + 1] = P.col_stat[1:prob.n + 1]
    Q.valid = 0
    assert Q.factorize() == 0 and Q.valid
    # B x = b through the factor glp_factorize built
    m = prob.m
    rng = np.random.default_rng(3)
    b = rng.standard_normal(m)
    B = np.zeros((m, m))                   # columns of (I | -A) for the basic variables
    for j in range(1, m + 1):
        k = Q.head[j]
        if k <= m:
            B[k - 1, j - 1] = 1.0
        else:
            lo, hi = prob.A_ptr[k - m - 1], prob.A_ptr[k - m]
            B[prob.A_ind[lo:hi] - 1, j - 1] = -prob.A_val[lo:hi]
    x = Q.ftran(b.copy())
    assert np.abs(B @ x - b).max() <= 1e-9 * max(1.0, np.abs(b).max())
    y = Q.ftran(b.copy(), tr=True)
    assert np.abs(B.T @ y - b).max() <= 1e-9 * max(1.0, np.abs(b).max())
    assert gk.glp_simplex(Q, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    R = gk.GkProblem(gpu_ctx, prob.copy())
    assert gk.glp_simplex(R, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    assert abs(Q.obj_val - R.obj_val) <= 1e-9 * max(1.0, abs(R.obj_val)), (Q.obj_val, R.obj_val)
    sparse_kkt(Q, prob)


def test_gpu_factor_choice_default(gpu_ctx, oracle, monkeypatch):
    """Without GK_SPARSE the factor follows the cost model (gk_engine.hip
    factor_choice): the block-angular m = 4,005 LP runs on the sparse LU and
    reaches the oracle's objective; C2s (m = 821) and dense A keep the
    explicit inverse."""
    monkeypatch.delenv("GK_SPARSE", raising=False)
    prob = problems.gen_blocks(40, 100, 200, 10)
    o = oracle.OracleProb(prob)
    assert o.simplex(meth=3) == 0
    ref = o.result()["obj_val"]
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    st = P.stats()
    assert st.factor_sparse == 1
    assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
    print(f"blocks 40 default: {P.it_cnt} pivots in {st.seconds_total:.2f} s ({P.it_cnt / st.seconds_total:.0f}/s), "
          f"host LU {st.seconds_lu:.2f} s")
    for prob in (problems.gen_c2s(), problems.gen_dense(256, 1024, seed=42)):
        Q = gk.GkProblem(gpu_ctx, prob)
        assert gk.glp_simplex(Q, gk.SMCP(meth=gk.GLP_DUAL, it_lim=50, msg_lev=gk.GLP_MSG_ERR)) in (0, 8)
        assert Q.stats().factor_sparse == 0


def test_gpu_warm_start_beyond_limit_default_factor(gpu_ctx, monkeypatch):
    """The path that hung in round 4, without GK_SPARSE: m > 65535, an
    it_lim solve, its statuses loaded into a new problem, glp_factorize of
    that advanced basis (the sparse factor by itself: the explicit m^2
    inverse is not built), FTRAN / BTRAN against scipy, then glp_simplex
    continuing from it."""
    import scipy.sparse as sps
    import scipy.sparse.linalg as spla
    monkeypatch.delenv("GK_SPARSE", raising=False)
    prob = problems.gen_blocks(656, 100, 200, 50)
    m = prob.m
    assert m > 65535
    P = gk.GkProblem(gpu_ctx, prob)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=1500, msg_lev=gk.GLP_MSG_ERR)) == problems.GLP_EITLIM
    Q = gk.GkProblem(gpu_ctx, prob.copy())
    Q.row_stat[1:m + 1] = P.row_stat[1:m + 1]
    Q.col_stat[1:prob.n + 1] = P.col_stat[1:prob.n + 1]
    Q.valid = 0
    assert Q.factorize() == 0 and Q.valid
    rows, cols, vals = [], [], []
    for j in range(1, m + 1):
        k = Q.head[j]
        if k <= m:
            rows.append(k - 1); cols.append(j - 1); vals.append(1.0)
        else:
            lo, hi = prob.A_ptr[k - m - 1], prob.A_ptr[k - m]
            rows += (np.asarray(prob.A_ind[lo:hi]) - 1).tolist()
            cols += [j - 1] * (hi - lo)
            vals += (-np.asarray(prob.A_val[lo:hi])).tolist()
    B = sps.csc_matrix((vals, (rows, cols)), shape=(m, m))
    b = np.random.default_rng(5).standard_normal(m)
    x = Q.ftran(b.copy())
    assert np.abs(B @ x - b).max() <= 1e-9 * max(1.0, np.abs(b).max())
    y = Q.ftran(b.copy(), tr=True)
    assert np.abs(B.T @ y - b).max() <= 1e-9 * max(1.0, np.abs(b).max())
    assert gk.glp_simplex(Q, gk.SMCP(meth=gk.GLP_DUAL, it_lim=500, msg_lev=gk.GLP_MSG_ERR)) == problems.GLP_EITLIM
    assert Q.stats().factor_sparse == 1
    check_solution(Q)


def test_gpu_tab_rows_on_sparse_factor(gpu_ctx, monkeypatch):
    """glp_eval_tab_row in a batch (gk_bfd_eval_tab_rows) on the sparse
    factor (rows of inv(B) by BTRANs): the rows the explicit inverse gives on
    the same optimal basis (glp_factorize of it each way), within 1e-9 of
    each row's largest entry."""
    prob = problems.gen_blocks(10, 100, 200, 5)
    P = gk.GkProblem(gpu_ctx, prob.copy())
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR)) == 0
    ks = [k for k in range(1, prob.m + prob.n + 1)
          if (P.row_stat[k] if k <= prob.m else P.col_stat[k - prob.m]) == problems.GLP_BS][:40]
    rows = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("GK_SPARSE", flag)
        Q = gk.GkProblem(gpu_ctx, prob.copy())
        Q.row_stat[1:prob.m + 1] = P.row_stat[1:prob.m + 1]
        Q.col_stat[1:prob.n + 1] = P.col_stat[1:prob.n + 1]
        Q.valid = 0
        assert Q.factorize() == 0
        rows[flag] = Q.eval_tab_rows(ks)
    a, b = rows["1"], rows["0"]
    big = np.maximum(1.0, np.abs(b).max(axis=1, keepdims=True))
    assert np.all(np.abs(a - b) <= 1e-9 * big)
