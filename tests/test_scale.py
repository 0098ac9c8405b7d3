"""glp_scale_prob (glpscl.js:1-225): the oracle restatement (oracle/scale.c)
against the reference's own factors, and the device path (gk_scale.hip)
against both, bit for bit.  The fixtures tests/golden/scale_*.json come from
the reference run by tests/golden/gen_golden.js (7 problems x 11 flag sets:
every flag alone, the combinations glp_simplex / glp_intopt use, AUTO, SKIP
and an invalid set), including the report lines the reference prints."""
import glob
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import orcpy  # noqa: E402

from glpk_js_amd import gk, problems  # noqa: E402

FIX = sorted(glob.glob(os.path.join(HERE, "golden", "scale_*.json")))


def _load(path):
    with open(path) as f:
        return json.load(f)


def _cases():
    for path in FIX:
        d = _load(path)
        for r in d["runs"]:
            yield pytest.param(path, r["flags"], id=f"{d['name']}-{r['flags']:#x}")


@pytest.mark.parametrize("path,flags", list(_cases()))
def test_oracle_scale_matches_reference(path, flags):
    d = _load(path)
    r = next(x for x in d["runs"] if x["flags"] == flags)
    ret, rii, sjj, rep = orcpy.scale_prob(d["m"], d["n"], d["A_ptr"], d["A_ind"], d["A_val"], flags)
    if "error" in r:
        assert ret == 1
        return
    assert ret == 0
    assert np.array_equal(rii, np.asarray(r["rii"], float))
    assert np.array_equal(sjj, np.asarray(r["sjj"], float))


def test_js_number_format():
    """the report lines print numbers as the reference's JS does"""
    for x, s in [(1.0, "1"), (10.0, "10"), (1.0000000000000002, "1.0000000000000002"),
                 (1.0071994140270092e-05, "0.000010071994140270092"), (3.1182412086163115e-10, "3.1182412086163115e-10"),
                 (19816686401.901344, "19816686401.901344"), (1e21, "1e+21"), (1e-7, "1e-7"), (2.5e-6, "0.0000025"),
                 (123456789012345680000.0, "123456789012345680000"), (-0.5, "-0.5")]:
        assert gk._js_num(x) == s, (x, s)


def _gpu_problem(ctx, d):
    m, n = d["m"], d["n"]
    p = problems.Problem(m=m, n=n, dir=problems.GLP_MIN, c0=0.0, name="",
                         row_type=np.full(m, problems.GLP_FR, np.int8), row_lb=np.zeros(m), row_ub=np.zeros(m),
                         rii=np.ones(m), row_stat=np.full(m, problems.GLP_BS, np.int8),
                         col_type=np.full(n, problems.GLP_FR, np.int8), col_lb=np.zeros(n), col_ub=np.zeros(n),
                         col_coef=np.zeros(n), sjj=np.ones(n), col_stat=np.full(n, problems.GLP_NS, np.int8),
                         col_kind=np.full(n, 1, np.int8), A_ptr=np.asarray(d["A_ptr"], np.int32),
                         A_ind=np.asarray(d["A_ind"], np.int32), A_val=np.asarray(d["A_val"], np.float64))
    return gk.GkProblem(ctx, p)


@pytest.mark.gpu
@pytest.mark.parametrize("path,flags", list(_cases()))
def test_gpu_scale_matches_reference(gpu_ctx, path, flags):
    """factors bit-identical to the reference's, and the same report lines"""
    d = _load(path)
    r = next(x for x in d["runs"] if x["flags"] == flags)
    P = _gpu_problem(gpu_ctx, d)
    lines = []
    gk.glp_set_print_func(lines.append)
    try:
        if "error" in r:
            with pytest.raises(gk.ScaleError) as ei:
                gk.glp_scale_prob(P, flags)
            assert str(ei.value) == r["error"]
            return
        gk.glp_scale_prob(P, flags)
    finally:
        gk.glp_set_print_func(None)
    assert np.array_equal(P.rii[1:d["m"] + 1], np.asarray(r["rii"], float))
    assert np.array_equal(P.sjj[1:d["n"] + 1], np.asarray(r["sjj"], float))
    assert lines == r["lines"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,m", [(1, 20000), (2, 20000), (3, 6000), (4, 8192)])
def test_gpu_scale_matches_oracle_large(gpu_ctx, seed, m):
    """larger random badly scaled matrices (empty rows and columns, magnitudes
    1e-6 .. 1e6) against the oracle, every flag combination the reference
    uses; m <= 8192 takes the LDS row-partials path, 20k rows the row copy"""
    rng = np.random.default_rng(seed)
    n, nnz = 30000, 300000
    rows = rng.integers(1, m + 1, nnz)
    rows[rows == 7] = 8                                   # an empty row
    cols = np.sort(rng.integers(0, n, nnz))
    cols[cols == 11] = 12                                 # an empty column
    vals = rng.choice([-1.0, 1.0], nnz) * 10.0 ** rng.integers(-6, 7, nnz) * (1 + rng.random(nnz))
    ptr = np.zeros(n + 1, np.int32)
    np.add.at(ptr, cols + 1, 1)
    ptr = np.cumsum(ptr).astype(np.int32)
    d = {"m": m, "n": n, "A_ptr": ptr, "A_ind": rows.astype(np.int32), "A_val": vals}
    P = _gpu_problem(gpu_ctx, d)
    gk.glp_set_print_func(lambda s: None)
    try:
        for flags in (0x31, 0x80, 0x01, 0x10, 0x21):
            ret, rii, sjj, _ = orcpy.scale_prob(m, n, ptr, d["A_ind"], vals, flags)
            assert ret == 0
            gk.glp_scale_prob(P, flags)
            assert np.array_equal(P.rii[1:m + 1], rii), flags
            assert np.array_equal(P.sjj[1:n + 1], sjj), flags
    finally:
        gk.glp_set_print_func(None)
