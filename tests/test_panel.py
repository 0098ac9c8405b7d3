"""MFMA panel pricing of the dual simplex's pivot row (gk_panel.hip).

In the column-pass regime (dense A, rho too dense for the row path) the
pivot row of eval_trow (glpspx02.js:655-791) comes from a panel of tableau
rows formed on the matrix cores and kept current by the product-form update;
the choice of the leaving row is the reference's chuzr, unchanged.  These
tests pin that the panel changes nothing the reference's results show:

  * forced onto the small dense fixtures (GK_PANEL_MIN_M=0; by default it
    engages from m = 1024), every dual run returns the reference's return
    code, statuses and objective, with panel sizes 32 and 2 (the latter
    refills on most pivots);
  * on the dense generator at 1024 x 4096 (default thresholds: the panel
    engages once the basis is half structural) the full dual solve has the
    reference's objective with and without the panel, both
    certified by KKT, and the panel served most pivot rows of its regime."""
import os

import pytest

from conftest import load_golden
from glpk_js_amd import gk, problems
from test_gpu_lp import LP_CASES, check_solution


def _dense_dual(c):
    d = load_golden(c.values[0])
    run = d["runs"][c.values[1]]
    if run["opts"].get("meth", 1) not in (gk.GLP_DUAL, gk.GLP_DUALP):
        return False
    p = problems.from_fixture(d)
    return p.m > 0 and p.n > 0 and len(p.A_val) >= 0.5 * p.m * p.n


DENSE_DUAL = [c for c in LP_CASES if _dense_dual(c)]


@pytest.fixture
def panel_env():
    keys = ("GK_PANEL", "GK_PANEL_MIN_M", "GK_PANEL_AGE")
    old = {k: os.environ.get(k) for k in keys}

    def set_(**kv):
        for k, v in kv.items():
            os.environ[k] = str(v)
    yield set_
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_panel_fixture_coverage():
    assert len(DENSE_DUAL) >= 6


@pytest.mark.gpu
@pytest.mark.parametrize("rows,age", [(32, 100), (2, 100), (32, 3)], ids=["32", "2", "32-age3"])
@pytest.mark.parametrize("path,run_index", DENSE_DUAL)
def test_gpu_panel_forced_matches_reference(gpu_ctx, panel_env, rows, age, path, run_index):
    """age 3: the panel is refilled whenever its rows went through three
    product-form updates, hit or not"""
    panel_env(GK_PANEL=rows, GK_PANEL_MIN_M=0, GK_PANEL_AGE=age)
    d = load_golden(path)
    run = d["runs"][run_index]
    P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
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


@pytest.mark.gpu
@pytest.mark.parametrize("age", [100, 1])
def test_gpu_panel_used_on_forced_fixture(gpu_ctx, panel_env, age):
    """the forced panel really serves the pivot rows (hits and refills
    counted by the device); at age 1 every pivot refills"""
    panel_env(GK_PANEL=32, GK_PANEL_MIN_M=0, GK_PANEL_AGE=age)
    used = hits = 0
    for c in DENSE_DUAL:
        d = load_golden(c.values[0])
        run = d["runs"][c.values[1]]
        P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
        gk.glp_simplex(P, gk.SMCP(**run["opts"]))
        st = P.stats()
        used += st.panel_hits + st.panel_refills
        hits += st.panel_hits
    assert used > 0
    if age == 1:
        assert hits == 0


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [32, 0], ids=["panel", "column-pass"])
def test_gpu_panel_dense_1024x4096_kkt(gpu_ctx, panel_env, rows):
    from kkt import dense_kkt
    panel_env(GK_PANEL=rows)
    prob = problems.gen_dense(1024, 4096, seed=42)
    P = gk.GkProblem(gpu_ctx, prob)
    hits = refills = 0
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=2000)
    while True:
        ret = gk.glp_simplex(P, parm)
        st = P.stats()
        hits += st.panel_hits
        refills += st.panel_refills
        if ret != 8:                      # GLP_EITLIM: continue from the basis left
            break
    assert ret == 0 and P.pbs_stat == P.dbs_stat == problems.GLP_FEAS
    ref = 978.22910129338311              # the reference's dual
    assert abs(P.obj_val - ref) <= 1e-9 * ref, P.obj_val
    dense_kkt(P, prob)
    if rows:
        assert hits > 0 and refills > 0
    else:
        assert hits == refills == 0
