"""The native LP / MIP presolver (gk_npp_*, glpk.js_amd/csrc/gk_npp.cc)
against the reference's glp_simplex and glp_intopt with presolve = GLP_ON
(glpapi06.js:41, glpapi09.js:116; mippre_* fixtures for the latter, with and
without binarize: npp_integer's binarization, hidden packing / covering and
coefficient reduction, glpnpp04.js).

Fixtures (tests/golden/gen_golden.js, presolveCase) record, per method, the
reduced problem the reference's npp_build_prob made (glpnpp01.js:396), the
solution of that problem its npp_postprocess received, and the final
solution.  On the CPU (host code, no device):

  * presolving the original problem gives the reference's return code, and
    when it goes on, the reduced problem bit for bit: row / column order and
    references, bounds, objective, constant term, every element in list
    order;
  * postprocessing the reference's solution of the reduced problem gives the
    reference's final statuses and values (bit for bit; the activities of
    basic rows to 1e-12, their sums run in the row-list order of the
    original problem, which the fixture does not carry).

On the GPU the whole glp_simplex(presolve = ON) flow runs: native presolve,
scaling and starting basis, device simplex, postprocessing (objective and
statuses against the reference)."""
import os

import numpy as np
import pytest

from conftest import golden_files, load_golden
from glpk_js_amd import problems

CASES = []
for path in golden_files("presolve_"):
    d = load_golden(path)
    for r, run in enumerate(d["runs"]):
        CASES.append(pytest.param(path, r, id=f"{os.path.basename(path)[9:-5]}-m{run['opts']['meth']}"))


def _presolve(d):
    from glpk_js_amd import presolve
    orig = problems.from_fixture(d)
    lp, arrays = presolve.problem_lp(orig)
    npp = presolve.Npp()
    npp.load(lp, None, presolve.GLP_SOL)
    return orig, lp, arrays, npp, npp.simplex()


@pytest.mark.parametrize("path,run_index", CASES)
def test_presolve_reduced_problem_matches_reference(path, run_index):
    d = load_golden(path)
    run = d["runs"][run_index]
    _, _, _, npp, ret = _presolve(d)
    red = run["reduced"]
    if red is None:
        # stopped by the preprocessor itself (glpapi06.js:69-84)
        assert ret == run["ret"]
        return
    assert ret == 0
    got = npp.build(d["dir"])
    assert (got.m, got.n, got.nnz) == (red["m"], red["n"], red["nnz"])
    assert list(npp.row_ref) == red["row_ref"] and list(npp.col_ref) == red["col_ref"]
    assert got.c0 == red["c0"]
    for key in ("row_type", "row_lb", "row_ub", "col_type", "col_lb", "col_ub", "col_coef"):
        np.testing.assert_array_equal(getattr(got, key), np.asarray(red[key]), err_msg=key)
    np.testing.assert_array_equal(got.A_ptr, np.asarray(red["A_ptr"]), err_msg="A_ptr")
    np.testing.assert_array_equal(got.A_ind, np.asarray(red["A_ind"]), err_msg="A_ind")
    np.testing.assert_array_equal(got.A_val, np.asarray(red["A_val"]), err_msg="A_val")


POST_CASES = [c for c in CASES if load_golden(c.values[0])["runs"][c.values[1]]["reduced_sol"] is not None]


@pytest.mark.parametrize("path,run_index", POST_CASES)
def test_postprocess_recovers_reference_solution(path, run_index):
    from glpk_js_amd import presolve
    d = load_golden(path)
    run = d["runs"][run_index]
    orig, lp, a, npp, ret = _presolve(d)
    assert ret == 0
    npp.build(d["dir"])
    s = run["reduced_sol"]
    pad = lambda v, t: np.concatenate([[0], np.asarray(v, t)]).astype(t)  # noqa: E731
    npp.postprocess_sol(s["pbs_stat"], s["dbs_stat"], pad(s["row_stat"], np.int8), pad(s["row_dual"], np.float64),
                        pad(s["col_stat"], np.int8), pad(s["col_prim"], np.float64))
    npp.L.gk_npp_unload_sol(npp.h, presolve.C.byref(lp))
    assert (lp.pbs_stat, lp.dbs_stat) == (run["pbs_stat"], run["dbs_stat"])
    np.testing.assert_array_equal(a["row_stat"][1:], run["row_stat"])
    np.testing.assert_array_equal(a["col_stat"][1:], run["col_stat"])
    np.testing.assert_array_equal(a["col_prim"][1:], np.asarray(run["col_prim"]), err_msg="col_prim")
    np.testing.assert_array_equal(a["row_dual"][1:], np.asarray(run["row_dual"]), err_msg="row_dual")
    for key in ("row_prim", "col_dual"):
        want = np.asarray(run[key], np.float64)
        assert np.max(np.abs(a[key][1:] - want), initial=0.0) <= 1e-12 * (1.0 + np.abs(want).max(initial=0.0)), key
    assert abs(lp.obj_val - run["obj_val"]) <= 1e-12 * max(1.0, abs(run["obj_val"]))


def test_presolve_fixture_coverage():
    """The fixtures exercise the preprocessor's outcomes: reduced problems
    solved to optimality, problems the preprocessor itself declares primal or
    dual infeasible, and reduced problems the solver finds infeasible."""
    rets, stopped, solved = set(), 0, 0
    for c in CASES:
        run = load_golden(c.values[0])["runs"][c.values[1]]
        rets.add(run["ret"])
        stopped += run["reduced"] is None
        solved += run["reduced_sol"] is not None
    assert {0, 10, 11} <= rets and stopped >= 10 and solved >= 40


@pytest.mark.gpu
@pytest.mark.parametrize("path,run_index", CASES)
def test_gpu_simplex_presolve_matches_reference(gpu_ctx, path, run_index):
    from glpk_js_amd import gk
    d = load_golden(path)
    run = d["runs"][run_index]
    P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
    ret = gk.glp_simplex(P, gk.SMCP(meth=run["opts"]["meth"], presolve=1))
    assert ret == run["ret"]
    if ret != 0:
        return
    assert (P.pbs_stat, P.dbs_stat) == (run["pbs_stat"], run["dbs_stat"])
    ref = run["obj_val"]
    assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
    from test_gpu_lp import check_solution
    check_solution(P)


# ---- glp_intopt with presolve = GLP_ON (glpapi09.js:116) -------------------
MIP_CASES = []
for path in golden_files("mippre_"):
    d = load_golden(path)
    for r, run in enumerate(d["runs"]):
        MIP_CASES.append(pytest.param(path, r, id=f"{os.path.basename(path)[7:-5]}-{'bin' if run['opts'].get('binarize') else 'nobin'}"))


def _presolve_mip(d, run):
    from glpk_js_amd import presolve
    orig = problems.from_fixture(d)
    lp, arrays = presolve.problem_lp(orig)
    npp = presolve.Npp()
    npp.load(lp, arrays["col_kind"], presolve.GLP_MIP)
    ret, msg = npp.integer(bool(run["opts"].get("binarize")))
    return orig, lp, arrays, npp, ret, msg


@pytest.mark.parametrize("path,run_index", MIP_CASES)
def test_mip_presolve_reduced_problem_matches_reference(path, run_index):
    d = load_golden(path)
    run = d["runs"][run_index]
    _, _, _, npp, ret, msg = _presolve_mip(d, run)
    red = run["reduced"]
    if red is None:
        assert ret == run["ret"]
        return
    assert ret == 0
    got = npp.build(d["dir"])
    assert (got.m, got.n, got.nnz) == (red["m"], red["n"], red["nnz"])
    assert list(npp.row_ref) == red["row_ref"] and list(npp.col_ref) == red["col_ref"]
    assert got.c0 == red["c0"]
    for key in ("row_type", "row_lb", "row_ub", "col_type", "col_lb", "col_ub", "col_coef", "col_kind"):
        np.testing.assert_array_equal(getattr(got, key), np.asarray(red[key]), err_msg=key)
    for key in ("A_ptr", "A_ind", "A_val"):
        np.testing.assert_array_equal(getattr(got, key), np.asarray(red[key]), err_msg=key)
    # the counts npp_integer prints (the reference's lines before the
    # reduced problem's size line)
    want = [s for s in run["lines"] if "were replaced by" in s or "row(s) were added" in s or
            "hidden packing" in s or "hidden covering" in s or "were reduced" in s or "Binarization failed" in s]
    made = []
    if msg[0] > 0:
        made.append(f"{msg[0]} integer variable(s) were replaced by {msg[1]} binary ones")
    if msg[2] > 0:
        made.append(f"{msg[2]} row(s) were added due to binarization")
    if msg[3] > 0:
        made.append(f"Binarization failed for {msg[3]} integer variable(s)")
    if msg[4] > 0:
        made.append(f"{msg[4]} hidden packing inequaliti(es) were detected")
    if msg[5] > 0:
        made.append(f"{msg[5]} hidden covering inequaliti(es) were detected")
    if msg[6] > 0:
        made.append(f"{msg[6]} constraint coefficient(s) were reduced")
    assert made == want


MIP_POST = [c for c in MIP_CASES if load_golden(c.values[0])["runs"][c.values[1]]["reduced_sol"] is not None]


@pytest.mark.parametrize("path,run_index", MIP_POST)
def test_mip_postprocess_recovers_reference_solution(path, run_index):
    from glpk_js_amd import presolve
    d = load_golden(path)
    run = d["runs"][run_index]
    orig, lp, a, npp, ret, _ = _presolve_mip(d, run)
    npp.build(d["dir"])
    s = run["reduced_sol"]
    npp.postprocess_mip(s["mip_stat"], np.concatenate([[0.0], np.asarray(s["col_mipx"], np.float64)]))
    st, obj = presolve.C.c_int(), presolve.C.c_double()
    f = presolve._ptr
    assert npp.L.gk_npp_unload_mip(npp.h, presolve.C.byref(lp), f(a["col_kind"]), f(a["row_mipx"]),
                                   f(a["col_mipx"]), presolve.C.byref(st), presolve.C.byref(obj)) == 0
    assert st.value == run["mip_stat"]
    np.testing.assert_array_equal(a["col_mipx"][1:], np.asarray(run["col_mipx"]))
    assert abs(obj.value - run["mip_obj"]) <= 1e-12 * max(1.0, abs(run["mip_obj"]))
    want = np.asarray(run["row_mipx"], np.float64)
    assert np.max(np.abs(a["row_mipx"][1:] - want), initial=0.0) <= 1e-12 * (1.0 + np.abs(want).max(initial=0.0))


@pytest.mark.gpu
@pytest.mark.parametrize("path,run_index", MIP_CASES)
def test_gpu_intopt_presolve_matches_reference(gpu_ctx, path, run_index):
    from glpk_js_amd import gk
    d = load_golden(path)
    run = d["runs"][run_index]
    P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
    lines = []
    gk.glp_set_print_func(lines.append)
    try:
        ret = gk.glp_intopt(P, gk.IOCP(**run["opts"]))
    finally:
        gk.glp_set_print_func(None)
    assert ret == run["ret"]
    assert P.mip_stat == run["mip_stat"]
    if P.mip_stat == gk.GLP_OPT:
        ref = run["mip_obj"]
        assert abs(P.mip_obj - ref) <= 1e-9 * max(1.0, abs(ref)), (P.mip_obj, ref)
    # the preprocessor's lines up to the LP relaxation (bit-exact text)
    cut = lambda ls: ls[:ls.index("Solving LP relaxation...")] if "Solving LP relaxation..." in ls else ls  # noqa: E731
    assert cut(lines) == cut(run["lines"])
