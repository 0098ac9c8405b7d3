"""GPU parity of the HIP simplex path (through the C-ABI) against the
reference's golden outputs and the oracle.

Bar (north star): objective within 1e-9 relative of the reference, identical
return codes and solution statuses.  Pivot sequences may differ where the GPU
reductions break near-ties differently, so iteration counts are only checked
where they are forced (it_lim runs)."""
import os

import numpy as np
import pytest

from conftest import golden_files, load_golden
from glpk_js_amd import gk, problems

pytestmark = pytest.mark.gpu

LP_CASES = []
for path in golden_files("lp_"):
    d = load_golden(path)
    for r, run in enumerate(d["runs"]):
        LP_CASES.append(pytest.param(path, r, id=f"{os.path.basename(path)[3:-5]}-{r}-m{run['opts'].get('meth', 1)}"))


def check_solution(P: gk.GkProblem, tol=1e-7):
    """Primal consistency of the stored solution: row activities equal A x,
    bounds hold within tolerance, objective equals c'x + c0."""
    p = P.p
    x = P.col_prim[1:]
    act = np.zeros(p.m)
    for j in range(p.n):
        lo, hi = p.A_ptr[j], p.A_ptr[j + 1]
        act[p.A_ind[lo:hi] - 1] += p.A_val[lo:hi] * x[j]
    scale = 1.0 + np.abs(act).max(initial=0.0)
    assert np.max(np.abs(act - P.row_prim[1:]), initial=0.0) <= 1e-8 * scale
    obj = p.c0 + float(np.dot(p.col_coef, x))
    assert abs(obj - P.obj_val) <= 1e-9 * max(1.0, abs(obj))


@pytest.mark.parametrize("path,run_index", LP_CASES)
def test_gpu_lp_matches_reference(gpu_ctx, path, run_index):
    d = load_golden(path)
    run = d["runs"][run_index]
    prob = problems.from_fixture(d)
    P = gk.GkProblem(gpu_ctx, prob)
    ret = gk.glp_simplex(P, gk.SMCP(**run["opts"]))
    assert ret == run["ret"]
    if run["opts"].get("it_lim"):
        assert P.it_cnt == run["it_cnt"]
        check_solution(P)
        return
    assert (P.pbs_stat, P.dbs_stat) == (run["pbs_stat"], run["dbs_stat"])
    if P.pbs_stat == problems.GLP_FEAS and P.dbs_stat == problems.GLP_FEAS:
        ref = run["obj_val"]
        assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
        check_solution(P)


IT_LIM_CASES = [c for c in LP_CASES if load_golden(c.values[0])["runs"][c.values[1]]["opts"].get("it_lim")]


@pytest.mark.parametrize("path,run_index", IT_LIM_CASES)
def test_gpu_lp_it_lim_state_matches_reference(gpu_ctx, path, run_index):
    """A run stopped by it_lim (glpspx01.js / glpspx02.js: ITERATION LIMIT
    EXCEEDED) leaves the reference's intermediate state: the same statuses,
    the same basis after it_lim pivots, and the same (non-optimal) objective
    and primal values.  The reference's pivot trace pins the pivots; a GPU
    run that followed them must reproduce this state exactly."""
    d = load_golden(path)
    run = d["runs"][run_index]
    prob = problems.from_fixture(d)
    P = gk.GkProblem(gpu_ctx, prob)
    ret = gk.glp_simplex(P, gk.SMCP(**run["opts"]))
    assert ret == run["ret"] and P.it_cnt == run["it_cnt"]
    assert (P.pbs_stat, P.dbs_stat) == (run["pbs_stat"], run["dbs_stat"])
    assert list(P.row_stat[1:]) == list(run["row_stat"])
    assert list(P.col_stat[1:]) == list(run["col_stat"])
    ref = run["obj_val"]
    assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
    for got, want in ((P.row_prim[1:], run["row_prim"]), (P.col_prim[1:], run["col_prim"])):
        want = np.asarray(want, np.float64)
        assert np.max(np.abs(np.asarray(got) - want), initial=0.0) <= 1e-9 * (1.0 + np.abs(want).max(initial=0.0))


@pytest.mark.parametrize("name", ["lp_gap.json", "lp_dense_64x256.json", "lp_mix14.json", "lp_c2s.json"])
def test_gpu_bfd_ftran_btran_match_oracle(gpu_ctx, oracle, name):
    """gk_bfd_factorize + gk_bfd_ftran/btran (glpapi12.js:5/:198/:222) agree
    with the oracle's LU+FT factor on the optimal basis of the instance."""
    d = load_golden(os.path.join(os.path.dirname(__file__), "golden", name))
    run = d["runs"][0]
    prob = problems.from_fixture(d)
    prob.row_stat = np.asarray(run["row_stat"], np.int8)
    prob.col_stat = np.asarray(run["col_stat"], np.int8)
    P = gk.GkProblem(gpu_ctx, prob)
    assert P.factorize() == 0
    o = oracle.OracleProb(prob)
    assert o.factorize() == 0
    rng = np.random.default_rng(1)
    for tr in (False, True):
        for _ in range(3):
            b = rng.standard_normal(prob.m)
            xg = P.ftran(b, tr=tr)
            xo = o.ftran(b, tr=tr)
            err = np.max(np.abs(xg - xo)) / (1.0 + np.max(np.abs(xo)))
            assert err <= 1e-10, err


def test_gpu_bfd_update_chain(gpu_ctx, oracle):
    """gk_bfd_update (bfd_update_it, glpbfd.js:170) over a chain of column
    replacements stays equal to a fresh factorization."""
    import ctypes as C
    prob = problems.gen_dense(48, 96, seed=3)
    P = gk.GkProblem(gpu_ctx, prob)
    assert P.factorize() == 0          # all-slack basis
    L = gk.load_library()
    m = prob.m
    Bcols = {i: (np.array([i], np.int32), np.array([1.0])) for i in range(1, m + 1)}
    rng = np.random.default_rng(5)
    pos = rng.permutation(m)[:20] + 1              # distinct positions and columns:
    cols = rng.permutation(prob.n)[:20]            # a repeated column would make B singular
    for t in range(20):
        j, c = int(pos[t]), int(cols[t])
        lo, hi = prob.A_ptr[c], prob.A_ptr[c + 1]
        ind = np.zeros(hi - lo + 1, np.int32); ind[1:] = prob.A_ind[lo:hi]
        val = np.zeros(hi - lo + 1); val[1:] = -prob.A_val[lo:hi]
        ret = L.gk_bfd_update(P.bfd, j, hi - lo, ind.ctypes.data_as(C.c_void_p), 0, val.ctypes.data_as(C.c_void_p))
        assert ret == 0
        Bcols[j] = (ind[1:].copy(), val[1:].copy())
    B = np.zeros((m, m))
    for j, (ind, val) in Bcols.items():
        B[ind - 1, j - 1] = val
    b = rng.standard_normal(m)
    y = np.zeros(m + 1); y[1:] = b
    L.gk_bfd_ftran(P.bfd, y.ctypes.data_as(C.c_void_p))
    x = np.linalg.solve(B, b)
    assert np.max(np.abs(y[1:] - x)) <= 1e-9 * (1 + np.max(np.abs(x)))
    assert L.gk_bfd_get_count(P.bfd) == 20


def test_gpu_dense_1024x4096_dual_matches_reference(gpu_ctx):
    """C3 proxy full solve; reference objective from SURVEY.md §4 (dual)."""
    prob = problems.gen_dense(1024, 4096, seed=42)
    P = gk.GkProblem(gpu_ctx, prob)
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL))
    assert ret == 0 and P.pbs_stat == P.dbs_stat == problems.GLP_FEAS
    ref = 978.22910129338311
    assert abs(P.obj_val - ref) <= 1e-9 * ref, P.obj_val
    check_solution(P)


def test_gpu_c3_full_size_iteration_limit(gpu_ctx):
    """C3 at full size (4096 x 16384): 300 dual pivots as the reference's
    it_lim=300 timing run; properties: EITLIM, exactly 300 pivots, the stored
    point satisfies A x = row activities, objective = c'x."""
    prob = problems.gen_dense(4096, 16384, seed=42)
    P = gk.GkProblem(gpu_ctx, prob)
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=300))
    assert ret == gk.GLP_EBOUND + 4     # GLP_EITLIM = 8
    assert P.it_cnt == 300
    check_solution(P)


def test_gpu_dense_2048x8192_full_dual_kkt(gpu_ctx):
    """A full dual solve of the dense generator at 2048 x 8192 (tens of
    thousands of pivots, re-inversions at k up to 2048); the returned basis
    is certified optimal by KKT (tests/kkt.py: feasibility, reduced costs,
    complementary slackness, zero duality gap within 1e-9), and its objective
    equals the oracle's full solve (tests/golden/dense_full_2048x8192.json,
    gen_dense_full_oracle.py) to 1e-9 relative."""
    from kkt import dense_kkt
    prob = problems.gen_dense(2048, 8192, seed=42)
    P = gk.GkProblem(gpu_ctx, prob)
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL))
    assert ret == 0 and P.pbs_stat == P.dbs_stat == problems.GLP_FEAS
    dense_kkt(P, prob)
    gold = os.path.join(os.path.dirname(__file__), "golden", "dense_full_2048x8192.json")
    ref = load_golden(gold)                        # the oracle's full solve (2.4 h on one core)
    assert abs(P.obj_val - ref["obj_val"]) <= 1e-9 * abs(ref["obj_val"]), (P.obj_val, ref)


def _gz(name):
    import gzip
    import json
    with gzip.open(os.path.join(os.path.dirname(__file__), "golden", name), "rt") as f:
        return json.load(f)


def _assert_state(P, want, tol=1e-9):
    """statuses equal; objective, primal and dual values within tol (relative
    to the vector's largest magnitude)"""
    assert (P.pbs_stat, P.dbs_stat) == (want["pbs_stat"], want["dbs_stat"])
    rs = np.asarray(P.row_stat[1:]) != np.asarray(want["row_stat"])
    cs = np.asarray(P.col_stat[1:]) != np.asarray(want["col_stat"])
    assert not rs.any() and not cs.any(), (f"{int(rs.sum())} row / {int(cs.sum())} column statuses differ; first "
                                           f"rows {np.nonzero(rs)[0][:5] + 1}, cols {np.nonzero(cs)[0][:5] + 1}")
    ref = want["obj_val"]
    assert abs(P.obj_val - ref) <= tol * max(1.0, abs(ref)), (P.obj_val, ref)
    for key in ("row_prim", "col_prim", "row_dual", "col_dual"):
        got, w = np.asarray(getattr(P, key)[1:]), np.asarray(want[key], np.float64)
        err = np.max(np.abs(got - w), initial=0.0)
        assert err <= tol * (1.0 + np.abs(w).max(initial=0.0)), (key, err)


@pytest.mark.parametrize("run_index", [0, 1], ids=["1x300", "3x100"])
def test_gpu_c3_full_size_state_matches_reference(gpu_ctx, run_index):
    """The headline instance at full size (C3 4096 x 16384, seed 42) against
    the reference itself: its 300-pivot timing run as one
    it_lim=300 call and as three it_lim=100 calls continuing from the basis
    the previous call left (the bench's step).  After 300 pivots the GPU holds
    the reference's basis (every row and column status), and its objective,
    primal and dual values agree to 1e-9 (tests/golden/c3_itlim.json.gz,
    gen_golden.js --c3)."""
    d = _gz("c3_itlim.json.gz")
    g, run = d["gen"], d["runs"][run_index]
    prob = problems.gen_dense(g["m"], g["n"], seed=g["seed"])
    P = gk.GkProblem(gpu_ctx, prob)
    for call in run["calls"]:
        ret = gk.glp_simplex(P, gk.SMCP(**run["opts"]))
        assert ret == call["ret"] and P.it_cnt == call["it_cnt"]
        assert abs(P.obj_val - call["obj_val"]) <= 1e-9 * max(1.0, abs(call["obj_val"])), (P.it_cnt, P.obj_val)
    _assert_state(P, run)
    check_solution(P)


def test_gpu_c3_bench_window_matches_oracle(gpu_ctx):
    """The bench's whole window on C3 (warm-up + timed steps: 25 calls of
    it_lim=100 from the slack basis, pivots 1-2500) against the oracle carried
    along the same calls (tests/golden/c3_oracle_window.json.gz; the oracle is
    bit-exact with the reference over the first 300 pivots,
    test_oracle_c3_full_size_matches_reference).  After every call the
    objective matches; at pivots 300 and 2500 the whole state does."""
    w = _gz("c3_oracle_window.json.gz")
    g = w["gen"]
    prob = problems.gen_dense(g["m"], g["n"], seed=g["seed"])
    P = gk.GkProblem(gpu_ctx, prob)
    states = {s["call"]: s for s in w["states"]}
    for k, want_ret in enumerate(w["rets"], start=1):
        ret = gk.glp_simplex(P, gk.SMCP(**w["opts"]))
        assert ret == want_ret and P.it_cnt == 100 * k
        if k in states:
            _assert_state(P, states[k])


@pytest.mark.gpu
def test_gpu_next_call_phase1_eval_bit_identical(gpu_ctx, monkeypatch):
    """A dual call stopped by it_lim in phase I evaluates the next call's
    phase-I basic values before it returns (gk_engine.hip next_aux_launch);
    the next call takes them only when nothing they depend on changed.  A
    chain of it_lim calls (with a bound changed between two of them) gives
    bit for bit the same states with the precomputation on and off
    (GK_NEXT_AUX=0), and the calls after an unchanged one do take it."""
    prob = problems.gen_dense(1024, 4096, seed=42)

    def chain(on):
        if on:
            monkeypatch.delenv("GK_NEXT_AUX", raising=False)
        else:
            monkeypatch.setenv("GK_NEXT_AUX", "0")
        P = gk.GkProblem(gpu_ctx, prob)
        out, skipped = [], 0
        for k in range(8):
            if k == 5:
                P.col_ub[7] = P.col_ub[7] + 0.5 if P.col_ub[7] < 1e30 else 10.0   # the next call rebuilds
            ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=60))
            skipped += P.stats().evals_skipped
            out.append((ret, P.it_cnt, P.obj_val, np.array(P.row_prim[1:]), np.array(P.col_prim[1:]),
                        np.array(P.row_stat[1:]), np.array(P.col_stat[1:])))
        return out, skipped

    on, sk_on = chain(True)
    off, sk_off = chain(False)
    for a, b in zip(on, off):
        assert a[:3] == b[:3]
        for x, y in zip(a[3:], b[3:]):
            assert np.array_equal(x, y)
    assert sk_on > sk_off


def test_gpu_bounds_version_fast_init_bit_identical(gpu_ctx):
    """gk_lp.b_version (ABI 8): a chain of it_lim calls with the bounds
    version declared (init_csa's arrays taken over from the resident working
    set, no rebuild, no comparison) ends bit for bit where the same chain with
    version 0 (rebuilt and compared every call) ends; a bound changed and
    declared with touch_bounds() is seen by the next call."""
    outs = []
    for declared in (False, True):
        prob = problems.gen_dense(256, 1024, seed=3)
        P = gk.GkProblem(gpu_ctx, prob)
        if declared:
            P.touch_bounds()
        trace = []
        for k in range(12):
            if k == 6:                      # a bound change in the middle of the chain
                P.row_ub[5] *= 0.5
                if declared:
                    P.touch_bounds()
            ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=40, msg_lev=gk.GLP_MSG_OFF))
            st = P.stats()
            trace.append((ret, P.it_cnt, P.obj_val, bytes(P.row_stat), bytes(P.col_stat),
                          (int(st.resident), int(st.evals_skipped), int(st.reinversions), int(st.refinements))))
        outs.append(trace)
    diag = [(k, a[:3] == b[:3], a[3] == b[3], a[4] == b[4], a[2].hex(), b[2].hex(), a[5], b[5])
            for k, (a, b) in enumerate(zip(*outs))]
    assert [a[:5] for a in outs[0]] == [b[:5] for b in outs[1]], diag


def test_gpu_end_of_call_epilogue_bit_identical(gpu_ctx, monkeypatch):
    """The end-of-call epilogue (gk_engine.hip Spx::epi_arm): the
    evaluations an it_lim call ends with, enqueued behind its last batch and
    gated on the batch's budget, give bit for bit the states of the host
    sequence (GK_EPILOGUE=0): a 1024 x 4096 chain through phase I with a bound
    changed in the middle and re-inversions inside calls, and a 512 x 2048
    chain to the optimum (batches that stop early leave the gated kernels
    doing nothing)."""
    def chain(prob, on, calls, change):
        monkeypatch.setenv("GK_EPILOGUE", "1" if on else "0")
        P = gk.GkProblem(gpu_ctx, prob)
        out, ret = [], 8
        for k in range(calls):
            if k == change:
                P.col_ub[7] = P.col_ub[7] + 0.5 if P.col_ub[7] < 1e30 else 10.0
            ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR))
            out.append((ret, P.it_cnt, float(P.obj_val).hex(), P.row_prim[1:].tobytes(), P.col_prim[1:].tobytes(),
                        P.row_dual[1:].tobytes(), P.col_dual[1:].tobytes(), bytes(P.row_stat[1:]),
                        bytes(P.col_stat[1:])))
            if ret != 8:
                break
        return out, ret

    big = problems.gen_dense(1024, 4096, seed=42)
    on, _ = chain(big, True, 60, 30)
    off, _ = chain(big, False, 60, 30)
    assert len(on) == len(off) == 60
    for k, (a, b) in enumerate(zip(on, off)):
        assert a == b, f"1024 x 4096, call {k} differs"
    small = problems.gen_dense(512, 2048, seed=7)          # 187 calls, 18,607 pivots to the optimum
    on, ret_on = chain(small, True, 400, -1)
    off, ret_off = chain(small, False, 400, -1)
    assert ret_on == ret_off == 0
    assert len(on) == len(off) > 100
    for k, (a, b) in enumerate(zip(on, off)):
        assert a == b, f"512 x 2048, call {k} differs"
