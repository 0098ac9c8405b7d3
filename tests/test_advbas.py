"""glp_adv_basis (glpini01.js:1): the triangular starting basis of the native
library (gk_adv_basis, host code) against the reference's own results on 16
problems (tests/golden/adv_*.json, written by gen_golden.js running the
reference): identical statuses and triangular-part size; and both simplex
methods run on the device from that basis return the reference's return
code, statuses and objective (<= 1e-9 relative).  The JS shim's rebinding of
glp_adv_basis is checked on the same fixtures by js/test_shim_cpu.js."""
import os
import re

import numpy as np
import pytest

from conftest import golden_files, load_golden
from glpk_js_amd import gk, problems

ADV = golden_files("adv_")


def test_fixtures_present():
    assert len(ADV) >= 10


@pytest.mark.parametrize("path", ADV, ids=[os.path.basename(p)[4:-5] for p in ADV])
def test_adv_basis_matches_reference(path):
    d = load_golden(path)
    size, rs, cs = gk.adv_basis_statuses(problems.from_fixture(d))
    np.testing.assert_array_equal(rs, np.asarray(d["adv"]["row_stat"], np.int8))
    np.testing.assert_array_equal(cs, np.asarray(d["adv"]["col_stat"], np.int8))
    m = [re.match(r"Size of triangular part = (\d+)", s) for s in d["adv"]["lines"]]
    m = [x for x in m if x]
    if d["m"] and d["n"]:
        assert size == int(m[0].group(1))
        # a basis: m basic variables
        assert int(np.sum(rs == problems.GLP_BS) + np.sum(cs == problems.GLP_BS)) == d["m"]


CASES = [pytest.param(p, r, id=f"{os.path.basename(p)[4:-5]}-m{load_golden(p)['runs'][r]['opts']['meth']}")
         for p in ADV for r in range(len(load_golden(p)["runs"]))]


@pytest.mark.gpu
@pytest.mark.parametrize("path,run_index", CASES)
def test_gpu_simplex_from_adv_basis(gpu_ctx, path, run_index):
    d = load_golden(path)
    run = d["runs"][run_index]
    if not (d["m"] and d["n"]):
        pytest.skip("no rows or columns: glp_simplex returns before the simplex")
    P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
    gk.glp_adv_basis(P, 0)
    ret = gk.glp_simplex(P, gk.SMCP(**run["opts"]))
    assert ret == run["ret"]
    assert (P.pbs_stat, P.dbs_stat) == (run["pbs_stat"], run["dbs_stat"])
    if P.pbs_stat == problems.GLP_FEAS and P.dbs_stat == problems.GLP_FEAS:
        ref = run["obj_val"]
        assert abs(P.obj_val - ref) <= 1e-9 * max(1.0, abs(ref)), (P.obj_val, ref)
