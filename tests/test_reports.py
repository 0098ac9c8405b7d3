"""The simplex driver's terminal output: the lines glp_simplex prints through
xprintf (glpapi06.js:325-328 header, glpspx01.js:1587 / glpspx02.js:1493-1495
display lines every out_frq pivots, the termination messages), recorded from
the reference by gen_golden.js in every lp_* fixture run.

CPU: every recorded display line and message is rebuilt from its fields by
gk.report_lines (the formatter the Python host applies to the engine's
gk_report_fn records, mirrored by js/gk_core.js reportLines) — string-equal,
which pins the JavaScript number formatting too.
GPU: glp_simplex on the device prints the reference's lines: identical text,
identical iteration numbers where the pivot count is the reference's, display
values within 1e-7 relative (sums over a basis computed by a different
factorization); where a near-tie broke differently the header and the
termination message still match."""
import math
import os
import re

import pytest

from conftest import golden_files, load_golden
from glpk_js_amd import gk, problems

PRIMAL = re.compile(r"^([ *])(\d+): obj = (\S+)  infeas = (\S+) \((\d+)\)$")
DUAL1 = re.compile(r"^ (\d+):  infeas = (\S+) \((\d+)\)$")
DUAL2 = re.compile(r"^\|(\d+): obj = (\S+)  infeas = (\S+) \((\d+)\)$")
INSTAB = re.compile(r"^Warning: numerical instability \((primal|dual) simplex, phase (I|II)\)$")

RUNS = [(p, r) for p in golden_files("lp_") + golden_files("adv_")
        for r, run in enumerate(load_golden(p)["runs"]) if "lines" in run]
LP_RUNS = [(p, r) for p, r in RUNS if os.path.basename(p).startswith("lp_")]


def _num(s):
    return {"Infinity": math.inf, "-Infinity": -math.inf, "NaN": math.nan}.get(s, None) or float(s)


def record_of(line):
    """The gk_report_fn record (kind, code, it, phase, obj, infeas, aux) a
    reference line corresponds to, or None for lines outside the engine."""
    m = PRIMAL.match(line)
    if m:
        return (1, 1, int(m[2]), 1 if m[1] == " " else 2, _num(m[3]), _num(m[4]), int(m[5]))
    m = DUAL1.match(line)
    if m:
        return (1, 2, int(m[1]), 1, 0.0, _num(m[2]), int(m[3]))
    m = DUAL2.match(line)
    if m:
        return (1, 2, int(m[1]), 2, _num(m[2]), _num(m[3]), int(m[4]))
    m = INSTAB.match(line)
    if m:
        return (2, 9, 0, 1 if m[2] == "I" else 2, 0.0, 0.0, 1 if m[1] == "primal" else 2)
    for code, text in gk._REPORT_MSG.items():
        if line == text:
            return (2, code, 0, 0, 0.0, 0.0, 0)
    return None


def test_fixtures_hold_lines():
    assert len(RUNS) >= 100


def test_report_lines_rebuild_reference_lines():
    seen = set()
    for path, r in RUNS:
        for line in load_golden(path)["runs"][r]["lines"]:
            rec = record_of(line)
            if rec is None:
                assert line.startswith(("GLPK Simplex Optimizer", "~")) or re.match(r"^\d+ rows?, ", line), line
                continue
            assert gk.report_lines(*rec) == [line]
            seen.add(rec[:2])
    # progress lines of both methods and several termination messages
    assert {(1, 1), (1, 2), (2, 1)} <= seen
    assert len({c for k, c in seen if k == 2}) >= 3


def test_factorization_error_lines():
    assert gk.report_lines(2, 11, 5, 2, 0.0, 0.0, 2) == [
        "Error: unable to factorize the basis matrix (2)", "Sorry, basis recovery procedure not implemented yet"]


def _lines_close(ours, ref):
    if len(ours) != len(ref):
        return False
    num = re.compile(r"-?(?:\d+\.?\d*(?:e[+-]?\d+)?|Infinity)")
    for a, b in zip(ours, ref):
        if num.sub("#", a) != num.sub("#", b):
            return False
        for x, y in zip(num.findall(a), num.findall(b)):
            fx, fy = _num(x), _num(y)
            if not abs(fx - fy) <= 1e-7 * max(1.0, abs(fy)):
                return False
    return True


@pytest.mark.gpu
@pytest.mark.parametrize("path,r", LP_RUNS, ids=[f"{os.path.basename(p)[3:-5]}-{r}" for p, r in LP_RUNS])
def test_gpu_simplex_prints_reference_lines(gpu_ctx, path, r):
    d = load_golden(path)
    run = d["runs"][r]
    P = gk.GkProblem(gpu_ctx, problems.from_fixture(d))
    lines = []
    gk.glp_set_print_func(lines.append)
    try:
        gk.glp_simplex(P, gk.SMCP(**run["opts"]))
    finally:
        gk.glp_set_print_func(None)
    ref = run["lines"]
    if P.it_cnt == run["it_cnt"]:
        assert _lines_close(lines, ref), (lines, ref)
    else:
        assert lines[:2] == ref[:2] and lines[-1] == ref[-1], (lines, ref)
