"""Problem instances for the simplex / branch-and-bound hot path.

A `Problem` holds exactly the fields of the reference problem object that the
hot path reads (glpapi01.js:1-35; init_csa in glpspx01.js:42-145): row and
column types, bounds, objective, scale factors, initial statuses and the
constraint matrix by columns *in column-list order* (A_ptr is 0-based, of
length n+1; A_ind holds 1-based row numbers, as lp.col[j].ptr walks them).

Generators reproduce SURVEY.md §8(d) exactly (splitmix64, seed 42): the dense
C3 family, the C2s sparse surrogate for netlib 25fv47, and the C5s correlated
multi-knapsack surrogate for mas76.  Matrices loaded with glp_load_matrix
(glpapi01.js:464) have every column list in descending row order, which the
generators replicate.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field

import numpy as np

# GLP_* constants (glpk.js:7-141)
GLP_MIN, GLP_MAX = 1, 2
GLP_CV, GLP_IV, GLP_BV = 1, 2, 3
GLP_FR, GLP_LO, GLP_UP, GLP_DB, GLP_FX = 1, 2, 3, 4, 5
GLP_BS, GLP_NL, GLP_NU, GLP_NF, GLP_NS = 1, 2, 3, 4, 5
GLP_UNDEF, GLP_FEAS, GLP_INFEAS, GLP_NOFEAS, GLP_OPT, GLP_UNBND = 1, 2, 3, 4, 5, 6
GLP_PRIMAL, GLP_DUALP, GLP_DUAL = 1, 2, 3
GLP_EFAIL, GLP_EOBJLL, GLP_EOBJUL, GLP_EITLIM, GLP_ETMLIM = 5, 6, 7, 8, 9

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix_uniform(seed: int, count: int, start: int = 0) -> np.ndarray:
    """Draws start+1 .. start+count of splitmix64(seed) as u = (z >> 11) * 2^-53."""
    with np.errstate(over="ignore"):
        k = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        s = np.uint64(seed) + k * _GAMMA
        z = s
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


class SplitMix:
    """Sequential splitmix64 stream (for generators with rejection sampling)."""

    def __init__(self, seed: int, block: int = 1 << 16):
        self.seed, self.pos, self.block = seed, 0, block
        self.buf = np.empty(0)
        self.i = 0

    def u(self) -> float:
        if self.i >= len(self.buf):
            self.buf = splitmix_uniform(self.seed, self.block, self.pos)
            self.pos += self.block
            self.i = 0
        v = self.buf[self.i]
        self.i += 1
        return float(v)


@dataclass
class Problem:
    m: int
    n: int
    dir: int
    c0: float
    row_type: np.ndarray
    row_lb: np.ndarray
    row_ub: np.ndarray
    rii: np.ndarray
    row_stat: np.ndarray
    col_type: np.ndarray
    col_lb: np.ndarray
    col_ub: np.ndarray
    col_coef: np.ndarray
    sjj: np.ndarray
    col_stat: np.ndarray
    col_kind: np.ndarray
    A_ptr: np.ndarray
    A_ind: np.ndarray
    A_val: np.ndarray
    name: str = ""
    dense: np.ndarray | None = field(default=None, repr=False)   # m x n column-major copy, if built dense

    @property
    def nnz(self) -> int:
        return int(self.A_ptr[-1])

    def copy(self) -> "Problem":
        kw = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in self.__dict__.items()}
        return Problem(**kw)


def _i8(a):
    return np.ascontiguousarray(a, dtype=np.int8)


def _f8(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i4(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _col_stat_for(col_type, col_lb, col_ub):
    """Status glp_set_col_bnds (glpapi01.js:247) gives a fresh non-basic column."""
    st = np.empty(len(col_type), dtype=np.int8)
    for j, t in enumerate(col_type):
        if t == GLP_FR:
            st[j] = GLP_NF
        elif t == GLP_LO:
            st[j] = GLP_NL
        elif t == GLP_UP:
            st[j] = GLP_NU
        elif t == GLP_DB:
            st[j] = GLP_NL if abs(col_lb[j]) <= abs(col_ub[j]) else GLP_NU
        else:
            st[j] = GLP_NS
    return st


def from_dense(a: np.ndarray, c: np.ndarray, b: np.ndarray, sense_max: bool, name: str = "",
               keep_dense: bool = True) -> Problem:
    """max/min c'x s.t. A x <= b (GLP_UP rows), x >= 0 (GLP_LO), glp_load_matrix order."""
    m, n = a.shape
    nnz_per_col = np.count_nonzero(a, axis=0)
    A_ptr = np.zeros(n + 1, dtype=np.int32)
    A_ptr[1:] = np.cumsum(nnz_per_col)
    if np.all(nnz_per_col == m):
        rows_desc = np.arange(m, 0, -1, dtype=np.int32)
        A_ind = np.tile(rows_desc, n)
        A_val = np.ascontiguousarray(a[::-1, :].T).reshape(-1)
    else:
        inds, vals = [], []
        for j in range(n):
            r = np.nonzero(a[:, j])[0][::-1]
            inds.append(r + 1)
            vals.append(a[r, j])
        A_ind = np.concatenate(inds).astype(np.int32)
        A_val = np.concatenate(vals)
    p = Problem(m=m, n=n, dir=GLP_MAX if sense_max else GLP_MIN, c0=0.0,
                row_type=_i8(np.full(m, GLP_UP)), row_lb=np.zeros(m), row_ub=_f8(b),
                rii=np.ones(m), row_stat=_i8(np.full(m, GLP_BS)),
                col_type=_i8(np.full(n, GLP_LO)), col_lb=np.zeros(n), col_ub=np.zeros(n),
                col_coef=_f8(c), sjj=np.ones(n), col_stat=_i8(np.full(n, GLP_NL)),
                col_kind=_i8(np.full(n, GLP_CV)), A_ptr=A_ptr, A_ind=_i4(A_ind), A_val=_f8(A_val),
                name=name)
    if keep_dense:
        p.dense = np.asfortranarray(a)
    return p


def gen_dense(m: int, n: int, seed: int = 42, keep_dense: bool = True) -> Problem:
    """C3 family: max sum c_j x_j, a_ij = 0.5 + u, rows <= 0.25 n."""
    c = splitmix_uniform(seed, n)
    a = 0.5 + splitmix_uniform(seed, m * n, start=n).reshape(m, n)
    b = np.full(m, 0.25 * n)
    return from_dense(a, c, b, True, name=f"dense_{m}x{n}", keep_dense=keep_dense)


def gen_c2s(m: int = 821, n: int = 1571, nzc: int = 7, seed: int = 42) -> Problem:
    """C2s surrogate for 25fv47: 7 distinct rows per column by rejection."""
    r = SplitMix(seed)
    c = np.array([r.u() for _ in range(n)])
    cols = []
    for _ in range(n):
        used, ent = set(), []
        while len(ent) < nzc:
            i = 1 + int(math.floor(r.u() * m))
            if i in used:
                continue
            used.add(i)
            ent.append((i, 0.5 + r.u()))
        cols.append(ent)
    b = np.array([1 + 9 * r.u() for _ in range(m)])
    A_ptr = np.zeros(n + 1, dtype=np.int32)
    inds, vals = [], []
    for j, ent in enumerate(cols):
        ent = sorted(ent, key=lambda t: -t[0])           # descending row order
        inds.extend(t[0] for t in ent)
        vals.extend(t[1] for t in ent)
        A_ptr[j + 1] = len(inds)
    return Problem(m=m, n=n, dir=GLP_MAX, c0=0.0,
                   row_type=_i8(np.full(m, GLP_UP)), row_lb=np.zeros(m), row_ub=_f8(b),
                   rii=np.ones(m), row_stat=_i8(np.full(m, GLP_BS)),
                   col_type=_i8(np.full(n, GLP_LO)), col_lb=np.zeros(n), col_ub=np.zeros(n),
                   col_coef=_f8(c), sjj=np.ones(n), col_stat=_i8(np.full(n, GLP_NL)),
                   col_kind=_i8(np.full(n, GLP_CV)), A_ptr=A_ptr, A_ind=_i4(inds), A_val=_f8(vals),
                   name=f"c2s_{m}x{n}")


def gen_c5s(m: int = 12, n: int = 30, seed: int = 42) -> Problem:
    """C5s correlated multi-knapsack surrogate for mas76."""
    u = splitmix_uniform(seed, m * n).reshape(m, n)
    w = 1.0 + np.floor(1000.0 * u)
    cap = np.floor(w.sum(axis=1) / 2.0)
    p = np.floor(w.sum(axis=0) / m) + 500.0
    prob = from_dense(w, p, cap, True, name=f"c5s_{m}x{n}", keep_dense=True)
    prob.col_type[:] = GLP_DB
    prob.col_lb[:] = 0.0
    prob.col_ub[:] = 1.0
    prob.col_kind[:] = GLP_IV
    prob.col_stat[:] = GLP_NL
    return prob


def from_fixture(d: dict) -> Problem:
    """Build the problem recorded by tests/golden/gen_golden.js."""
    gen = d.get("gen")
    if gen:
        kind = gen["kind"]
        if kind == "dense":
            p = gen_dense(gen["m"], gen["n"], gen["seed"])
        elif kind == "c2s":
            p = gen_c2s(gen["m"], gen["n"], gen["nzc"], gen["seed"])
        elif kind == "c5s":
            p = gen_c5s(gen["m"], gen["n"], gen["seed"])
        else:
            raise ValueError(kind)
    else:
        p = Problem(m=d["m"], n=d["n"], dir=d["dir"], c0=float(d["c0"]),
                    row_type=_i8(d["row_type"]), row_lb=_f8(d["row_lb"]), row_ub=_f8(d["row_ub"]),
                    rii=_f8(d["row_rii"]), row_stat=_i8(d["row_stat"]),
                    col_type=_i8(d["col_type"]), col_lb=_f8(d["col_lb"]), col_ub=_f8(d["col_ub"]),
                    col_coef=_f8(d["col_coef"]), sjj=_f8(d["col_sjj"]), col_stat=_i8(d["col_stat"]),
                    col_kind=_i8(d["col_kind"]), A_ptr=_i4(d["A_ptr"]), A_ind=_i4(d["A_ind"]),
                    A_val=_f8(d["A_val"]), name=d.get("name", ""))
    # statuses/bounds exactly as recorded (covers kinds set by glp_set_col_kind)
    for key, conv in (("row_type", _i8), ("row_lb", _f8), ("row_ub", _f8), ("row_stat", _i8),
                      ("col_type", _i8), ("col_lb", _f8), ("col_ub", _f8), ("col_coef", _f8),
                      ("col_stat", _i8), ("col_kind", _i8)):
        if key in d:
            setattr(p, key, conv(d[key]))
    p.name = d.get("name", p.name)
    return p


def load_fixture(path: str) -> dict:
    with open(path) as f:
        return json.load(f)
