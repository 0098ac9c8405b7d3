"""Run-to-run determinism of the device simplex: the same input gives the
same pivot path, bit for bit.

Round 4's C3 dual solve took 381,770 pivots in one run and 380,308 in the
next (2 against 5 "numerical instability" recoveries): the writer block of
several multi-block pivot kernels stored scalar state that other blocks of
the same launch still had to read, and blocks start on the 8 XCDs
independently (gk_device.h, gate_arrive / gate_wait).  These tests pin the
fix: repeated solves agree in every batch's state fingerprint (the engine's
GK_DET_LOG: hashes of the header, statuses, basic values, reduced costs,
weights and inv(B) after every batch and re-inversion), in the iteration
and re-inversion counts and in the returned solution's bits."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402


def _solve(ctx, prob, it_lim=None):
    P = gk.GkProblem(ctx, prob)
    kw = {"it_lim": it_lim} if it_lim else {}
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR, **kw))
    st = P.stats()
    r = P.result()
    out = {"ret": ret, "it_cnt": P.it_cnt, "obj": float(P.obj_val).hex(), "reinversions": st.reinversions,
           "refinements": st.refinements, "row_stat": r["row_stat"].tobytes(), "col_stat": r["col_stat"].tobytes(),
           "row_prim": np.asarray(r["row_prim"]).tobytes(), "col_dual": np.asarray(r["col_dual"]).tobytes()}
    del P
    return out


@pytest.mark.gpu
def test_gpu_dense_1024x4096_full_dual_repeatable():
    """Three full dual solves of the 1024x4096 generator in one process: the
    same return code, pivot count, re-inversion counts, objective bits and
    primal / dual values bit for bit (and the reference's objective)."""
    ctx = gk.Context(0)
    prob = problems.gen_dense(1024, 4096, seed=42)
    runs = [_solve(ctx, prob) for _ in range(3)]
    assert runs[0]["ret"] == 0
    assert abs(float.fromhex(runs[0]["obj"]) - 978.22910129338311) <= 1e-9 * 978.2291
    for r in runs[1:]:
        assert r == runs[0]


@pytest.mark.gpu
def test_gpu_c3_dual_30k_pivots_fingerprints_repeatable(tmp_path):
    """C3 (4096 x 16384) dual from the slack basis through 30,000 pivots,
    twice in one process and once more in a second process: every batch's
    state fingerprint (GK_DET_LOG) equal, no instability recovery printed."""
    log = tmp_path / "det.log"
    env = dict(os.environ, GK_DET_LOG=str(log))
    outs = []
    for reps in (2, 1):
        r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "det_probe.py"), "4096", "16384",
                            "30000", str(reps)], capture_output=True, text=True, env=env, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "numerical instability" not in r.stdout + r.stderr
        outs += [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(outs) == 3 and len({(o["it_cnt"], o["obj"], o["reinversions"]) for o in outs}) == 1, outs
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import det_probe
    runs = det_probe.runs_of(str(log))
    assert len(runs) == 3 and len(runs[0]) > 300
    assert runs[1] == runs[0] and runs[2] == runs[0], "\n".join(det_probe.compare(runs))
