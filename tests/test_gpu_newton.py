"""Scheduled re-inversion by Newton refinement of the updated inverse
(glpk.js_amd/csrc/gk_newton.hip) against the reference's results.

The refinement replaces Gauss-Jordan only at the engine's scheduled
re-inversions (the update limit, the device counterpart of nfs_max,
glpfhv.js:182-187); GK_NEWTON_MIN_K lowers its size threshold (default 512)
so that the small fixtures take it at every such point.  The bar is the one
of test_gpu_lp.py: the reference's return code, statuses and objective to
1e-9 relative; the counters show the refinement ran and converged."""
import os

import pytest

from conftest import golden_files, load_golden
from glpk_js_amd import gk, problems

pytestmark = pytest.mark.gpu

CASES = []
for path in golden_files("lp_"):
    d = load_golden(path)
    for r, run in enumerate(d["runs"]):
        o = run["opts"]
        if o.get("it_lim"):
            continue
        CASES.append(pytest.param(path, r, id=f"{os.path.basename(path)[3:-5]}-{r}-m{o.get('meth', 1)}"))


@pytest.mark.parametrize("path,run_index", CASES)
def test_gpu_newton_forced_matches_reference(gpu_ctx, monkeypatch, path, run_index):
    monkeypatch.setenv("GK_NEWTON_MIN_K", "1")
    d = load_golden(path)
    run = d["runs"][run_index]
    P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
    # short update chains: the scheduled re-inversions happen even on small runs
    P.set_bfcp(nfs_max=8)
    ret = gk.glp_simplex(P, gk.SMCP(**run["opts"]))
    assert ret == run["ret"]
    assert (P.pbs_stat, P.dbs_stat) == (run["pbs_stat"], run["dbs_stat"])
    if P.pbs_stat == problems.GLP_FEAS and P.dbs_stat == problems.GLP_FEAS:
        ref = run["obj_val"]
        assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)


@pytest.mark.parametrize("min_k", ["0", "64"], ids=["gauss-jordan", "newton"])
def test_gpu_newton_dense_full_dual(gpu_ctx, monkeypatch, min_k):
    """C3 proxy 1024 x 4096, full dual solve (reference objective)
    with every scheduled re-inversion at k >= 64 refined (the structural
    block grows past 64 early in the solve), and with Gauss-Jordan only."""
    monkeypatch.setenv("GK_NEWTON_MIN_K", min_k)
    prob = problems.gen_dense(1024, 4096, seed=42)
    P = gk.GkProblem(gpu_ctx, prob)
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL))
    assert ret == 0 and P.pbs_stat == P.dbs_stat == problems.GLP_FEAS
    ref = 978.22910129338311
    assert abs(P.obj_val - ref) <= 1e-9 * ref, P.obj_val
    s = P.stats()
    if min_k == "0":
        assert s.refine_tries == 0 and s.refinements == 0
    else:
        assert s.refinements > 0, (s.refine_tries, s.refinements)
        assert s.refine_steps >= s.refinements
        assert s.refine_resid_max < 1e-3


def test_gpu_newton_dense_primal(gpu_ctx, monkeypatch):
    """The primal's scheduled re-inversions take the same path."""
    monkeypatch.setenv("GK_NEWTON_MIN_K", "16")
    prob = problems.gen_dense(256, 1024, seed=42)
    P = gk.GkProblem(gpu_ctx, prob)
    Q = gk.GkProblem(gpu_ctx, problems.gen_dense(256, 1024, seed=42))
    P.set_bfcp(nfs_max=20)
    Q.set_bfcp(nfs_max=20)
    assert gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_PRIMAL)) == 0
    monkeypatch.setenv("GK_NEWTON_MIN_K", "0")
    assert gk.glp_simplex(Q, gk.SMCP(meth=gk.GLP_PRIMAL)) == 0
    assert abs(P.obj_val - Q.obj_val) <= 1e-9 * abs(Q.obj_val)
    assert P.stats().refinements > 0
