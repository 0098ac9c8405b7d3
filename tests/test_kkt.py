"""The KKT certificate (tests/kkt.py) used for full-size GPU solves, checked
on the oracle's optimal solutions of the dense generator (CPU), and shown to
reject a perturbed (non-optimal) solution."""
import numpy as np
import pytest

from glpk_js_amd import problems
from kkt import dense_kkt


class _Sol:
    def __init__(self, r):
        self.col_prim = np.r_[0.0, r["col_prim"]]
        self.col_dual = np.r_[0.0, r["col_dual"]]
        self.row_prim = np.r_[0.0, r["row_prim"]]
        self.row_dual = np.r_[0.0, r["row_dual"]]
        self.obj_val = r["obj_val"]


@pytest.mark.parametrize("m,n", [(64, 256), (128, 512)])
def test_kkt_certifies_oracle_optimum(oracle, m, n):
    p = problems.gen_dense(m, n, seed=42)
    o = oracle.OracleProb(p)
    assert o.simplex(meth=3) == 0
    dense_kkt(_Sol(o.result()), p)


def test_kkt_rejects_suboptimal_point(oracle):
    p = problems.gen_dense(64, 256, seed=42)
    o = oracle.OracleProb(p)
    assert o.simplex(meth=3, it_lim=20) == 8         # stopped early: not optimal
    with pytest.raises(AssertionError):
        dense_kkt(_Sol(o.result()), p)
