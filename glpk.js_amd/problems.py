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


def gen_blocks(blocks: int = 1000, mb: int = 100, nb: int = 200, links: int = 50, nzc: int = 7,
               seed: int = 42) -> Problem:
    """Block-angular sparse LP (the sparse factor path's large instance, DESIGN
    §2f): `blocks` independent C2s-like blocks of mb rows x nb columns (nzc
    distinct rows of its block per column, drawn by rejection, a = 0.5 + u)
    plus `links` linking rows, column j entering linking row j mod links with
    0.5 + u.  Maximize c'x (c_j = u), block rows <= 1 + 9u, linking rows
    <= 0.25 blocks mb / links, x >= 0.  splitmix64 in the order c, then per
    column its rows and values, then the block bounds.  m = blocks mb + links,
    n = blocks nb; the default is m = 100,050, n = 200,000."""
    r = SplitMix(seed)
    m, n = blocks * mb + links, blocks * nb
    c = np.array([r.u() for _ in range(n)])
    A_ptr = np.zeros(n + 1, dtype=np.int32)
    inds, vals = [], []
    for j in range(n):
        k = j // nb
        used, ent = set(), []
        while len(ent) < nzc:
            i = k * mb + 1 + int(math.floor(r.u() * mb))
            if i in used:
                continue
            used.add(i)
            ent.append((i, 0.5 + r.u()))
        ent.append((blocks * mb + 1 + j % links, 0.5 + r.u()))
        ent.sort(key=lambda t: -t[0])                    # descending row order (glp_load_matrix)
        inds.extend(t[0] for t in ent)
        vals.extend(t[1] for t in ent)
        A_ptr[j + 1] = len(inds)
    b = np.concatenate([np.array([1 + 9 * r.u() for _ in range(blocks * mb)]),
                        np.full(links, 0.25 * blocks * mb / links)])
    return Problem(m=m, n=n, dir=GLP_MAX, c0=0.0,
                   row_type=_i8(np.full(m, GLP_UP)), row_lb=np.zeros(m), row_ub=_f8(b),
                   rii=np.ones(m), row_stat=_i8(np.full(m, GLP_BS)),
                   col_type=_i8(np.full(n, GLP_LO)), col_lb=np.zeros(n), col_ub=np.zeros(n),
                   col_coef=_f8(c), sjj=np.ones(n), col_stat=_i8(np.full(n, GLP_NL)),
                   col_kind=_i8(np.full(n, GLP_CV)), A_ptr=A_ptr, A_ind=_i4(inds), A_val=_f8(vals),
                   name=f"blocks_{blocks}x{mb}x{nb}+{links}")


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


# ---------------------------------------------------------------------------
# CPLEX LP format reader (glp_read_lp, glpcpx.js:10-753): the problem as the
# reference builds it — columns in order of first appearance, column lists
# sorted by row (glp_sort_matrix), bounds stored as glp_set_col_bnds stores
# them, zero coefficients dropped, binaries as integer columns with 0-1 bounds
# ---------------------------------------------------------------------------
_LP_CHARSET = "!\"#$%&()/,.;?@_`'{}|~"
_LP_KEYWORDS = {"minimize": "min", "minimum": "min", "min": "min", "maximize": "max", "maximum": "max",
                "max": "max", "st": "st", "s.t.": "st", "st.": "st", "bounds": "bounds", "bound": "bounds",
                "general": "gen", "generals": "gen", "gen": "gen", "integer": "int", "integers": "int",
                "int": "int", "binary": "bin", "binaries": "bin", "bin": "bin", "end": "end"}


class LpFormatError(ValueError):
    pass


def _lp_tokens(text: str):
    """Tokens (kind, image, value, next_char, line) with glp_read_lp's rules:
    keywords only at the start of a line, '\\' comments, '<', '<=', '=<', ..."""
    s = text if text.endswith("\n") else text + "\n"
    i, line, at_line_start = 0, 1, True
    out = []
    N = len(s)

    def isname(ch):
        return ch.isalnum() or ch in _LP_CHARSET

    while True:
        while i < N and s[i] != "\n" and s[i].isspace():
            i += 1
        if i >= N:
            out.append(("eof", "", 0.0, "", line))
            return out
        ch = s[i]
        if ch == "\n":
            i += 1
            line += 1
            at_line_start = True
            continue
        if ch == "\\":
            while i < N and s[i] != "\n":
                i += 1
            continue
        start_of_line = at_line_start
        at_line_start = False
        if ch.isalpha() or (ch != "." and ch in _LP_CHARSET):
            j = i
            while j < N and isname(s[j]):
                j += 1
            img = s[i:j]
            kind = "name"
            if start_of_line:
                low = img.lower()
                if low in ("subject", "such"):
                    k = j
                    if k < N and s[k] == " ":
                        k2 = k + 1
                        want = "to" if low == "subject" else "that"
                        if s[k2:k2 + len(want)].lower() == want and not (k2 + len(want) < N and s[k2 + len(want)].isalpha()):
                            kind, img, j = "st", s[i:k2 + len(want)], k2 + len(want)
                elif low in _LP_KEYWORDS:
                    kind = _LP_KEYWORDS[low]
            i = j
            out.append((kind, img, 0.0, _lp_peek(s, i), line))
            continue
        if ch.isdigit() or ch == ".":
            j = i
            while j < N and s[j].isdigit():
                j += 1
            if j < N and s[j] == ".":
                j += 1
                if j - i == 1 and not (j < N and s[j].isdigit()):
                    raise LpFormatError(f"{line}: invalid use of decimal point")
                while j < N and s[j].isdigit():
                    j += 1
            if j < N and s[j] in "eE":
                j += 1
                if j < N and s[j] in "+-":
                    j += 1
                if not (j < N and s[j].isdigit()):
                    raise LpFormatError(f"{line}: numeric constant `{s[i:j]}' incomplete")
                while j < N and s[j].isdigit():
                    j += 1
            img = s[i:j]
            i = j
            out.append(("num", img, float(img), _lp_peek(s, i), line))
            continue
        if ch in "+-:":
            i += 1
            out.append(({"+": "plus", "-": "minus", ":": "colon"}[ch], ch, 0.0, _lp_peek(s, i), line))
            continue
        if ch in "<>=":
            j = i + 1
            kind = {"<": "le", ">": "ge", "=": "eq"}[ch]
            if ch in "<>" and j < N and s[j] == "=":
                j += 1
            elif ch == "=" and j < N and s[j] in "<>":
                kind = "le" if s[j] == "<" else "ge"
                j += 1
            img = s[i:j]
            i = j
            out.append((kind, img, 0.0, _lp_peek(s, i), line))
            continue
        raise LpFormatError(f"{line}: character `{ch}' not recognized")


def _lp_peek(s: str, i: int) -> str:
    """the next significant character after a token (blanks skipped), as
    glp_read_lp sees csa.c after scan_token"""
    while i < len(s) and s[i] != "\n" and s[i].isspace():
        i += 1
    return s[i] if i < len(s) else ""


def read_lp(text: str) -> Problem:
    """glp_read_lp (glpcpx.js:10) on the text of a CPLEX LP file."""
    toks = _lp_tokens(text)
    pos = 0
    cols: dict[str, int] = {}
    col_names: list[str] = []
    lbs: list[float] = []
    ubs: list[float] = []
    obj: dict[int, float] = {}
    isint: set[int] = set()
    rows: list[tuple[list[int], list[float], int, float]] = []
    BIG = 1.7976931348623157e308

    def tok():
        return toks[pos]

    def nxt():
        nonlocal pos
        pos += 1

    def err(msg):
        raise LpFormatError(f"{tok()[4]}: {msg}")

    def find_col(name):
        if name not in cols:
            cols[name] = len(col_names)
            col_names.append(name)
            lbs.append(+BIG)
            ubs.append(-BIG)
        return cols[name]

    def linear_form():
        ind, val, used = [], [], set()
        while True:
            s = 1.0
            if tok()[0] in ("plus", "minus"):
                s = 1.0 if tok()[0] == "plus" else -1.0
                nxt()
            coef = 1.0
            if tok()[0] == "num":
                coef = tok()[2]
                nxt()
            if tok()[0] != "name":
                err("missing variable name")
            j = find_col(tok()[1])
            if j in used:
                err(f"multiple use of variable `{tok()[1]}' not allowed")
            used.add(j)
            ind.append(j)
            val.append(s * coef)
            nxt()
            if tok()[0] in ("plus", "minus"):
                continue
            keep = [(a, v) for a, v in zip(ind, val) if v != 0.0]
            return [a for a, _ in keep], [v for _, v in keep]

    # objective
    if tok()[0] not in ("min", "max"):
        err("`minimize' or `maximize' keyword missing")
    direction = GLP_MIN if tok()[0] == "min" else GLP_MAX
    nxt()
    if tok()[0] == "name" and tok()[3] == ":":
        nxt()
        nxt()
    ind, val = linear_form()
    for a, v in zip(ind, val):
        obj[a] = v
    # constraints
    if tok()[0] != "st":
        err("constraints section missing")
    nxt()
    while True:
        if tok()[0] == "name" and tok()[3] == ":":
            nxt()
            nxt()
        ind, val = linear_form()
        kind = tok()[0]
        if kind == "le":
            rtype = GLP_UP
        elif kind == "ge":
            rtype = GLP_LO
        elif kind == "eq":
            rtype = GLP_FX
        else:
            err("missing constraint sense")
        nxt()
        s = 1.0
        if tok()[0] in ("plus", "minus"):
            s = 1.0 if tok()[0] == "plus" else -1.0
            nxt()
        if tok()[0] != "num":
            err("missing right-hand side")
        rows.append((ind, val, rtype, s * tok()[2]))
        if tok()[3] not in ("\n", ""):
            err("invalid symbol(s) beyond right-hand side")
        nxt()
        if tok()[0] in ("plus", "minus", "num", "name"):
            continue
        break
    # bounds
    if tok()[0] == "bounds":
        nxt()
        while tok()[0] in ("plus", "minus", "num", "name"):
            lb_flag, lb = False, 0.0
            if tok()[0] in ("plus", "minus"):
                s = 1.0 if tok()[0] == "plus" else -1.0
                nxt()
                lb_flag = True
                if tok()[0] == "num":
                    lb = s * tok()[2]
                    nxt()
                elif tok()[1].lower() in ("infinity", "inf"):
                    if s > 0:
                        err("invalid use of `+inf' as lower bound")
                    lb = -BIG
                    nxt()
                else:
                    err("missing lower bound")
            elif tok()[0] == "num":
                lb_flag, lb = True, tok()[2]
                nxt()
            if lb_flag:
                if tok()[0] != "le":
                    err("missing `<', `<=', or `=<' after lower bound")
                nxt()
            if tok()[0] != "name":
                err("missing variable name")
            j = find_col(tok()[1])
            if lb_flag:
                lbs[j] = lb
            nxt()
            k = tok()[0]
            if k in ("le", "ge", "eq"):
                if k != "le" and lb_flag:
                    err("invalid bound definition")
                nxt()
                s = 1.0
                signed = tok()[0] in ("plus", "minus")
                if signed:
                    s = 1.0 if tok()[0] == "plus" else -1.0
                    nxt()
                if tok()[0] == "num":
                    v = s * tok()[2]
                    if k == "le":
                        ubs[j] = v
                    elif k == "ge":
                        lbs[j] = v
                    else:
                        lbs[j] = ubs[j] = v
                    nxt()
                elif signed and k == "le" and tok()[1].lower() in ("infinity", "inf"):
                    if s < 0:
                        err("invalid use of `-inf' as upper bound")
                    ubs[j] = +BIG
                    nxt()
                elif signed and k == "ge" and (tok()[1].lower() == "infinity" or tok()[1].lower() != "inf"):
                    # as the reference: any token but `inf' reads as infinity
                    # after `>= -' (glpcpx.js:543, `the_same(...) == 0')
                    if s > 0:
                        err("invalid use of `+inf' as lower bound")
                    lbs[j] = -BIG
                    nxt()
                elif k == "le":
                    err("missing upper bound")
                elif k == "ge":
                    err("missing lower bound")
                else:
                    err("missing fixed value")
            elif tok()[0] == "name" and tok()[1].lower() == "free":
                if lb_flag:
                    err("invalid bound definition")
                lbs[j], ubs[j] = -BIG, +BIG
                nxt()
            elif not lb_flag:
                err("invalid bound definition")
    # general / integer / binary
    while tok()[0] in ("gen", "int", "bin"):
        binary = tok()[0] == "bin"
        nxt()
        while tok()[0] == "name":
            j = find_col(tok()[1])
            isint.add(j)
            if binary:
                lbs[j], ubs[j] = 0.0, 1.0
            nxt()
    if tok()[0] == "end":
        nxt()
    elif tok()[0] != "eof":
        err(f"symbol {tok()[1]} in wrong position")
    if tok()[0] != "eof":
        err("extra symbol(s) detected beyond `end'")
    # columns: bounds as glp_set_col_bnds stores them, statuses of non-basic columns
    n, m = len(col_names), len(rows)
    ctype, clb, cub, cstat = [], [], [], []
    for j in range(n):
        lb = 0.0 if lbs[j] == +BIG else lbs[j]
        ub = +BIG if ubs[j] == -BIG else ubs[j]
        if lb == -BIG and ub == +BIG:
            t, l, u, st = GLP_FR, 0.0, 0.0, GLP_NF
        elif ub == +BIG:
            t, l, u, st = GLP_LO, lb, 0.0, GLP_NL
        elif lb == -BIG:
            t, l, u, st = GLP_UP, 0.0, ub, GLP_NU
        elif lb != ub:
            t, l, u, st = GLP_DB, lb, ub, GLP_NL
        else:
            t, l, u, st = GLP_FX, lb, ub, GLP_NS
        ctype.append(t); clb.append(l); cub.append(u); cstat.append(st)
    rtype, rlb, rub = [], [], []
    for (_, _, t, rhs) in rows:
        rtype.append(t)
        rlb.append(0.0 if t == GLP_UP else rhs)
        rub.append(0.0 if t == GLP_LO else rhs)
    # column lists sorted by row (glp_sort_matrix)
    entries = [[] for _ in range(n)]
    for i, (ind, val, _, _) in enumerate(rows):
        for a, v in zip(ind, val):
            entries[a].append((i + 1, v))
    A_ptr = np.zeros(n + 1, np.int32)
    A_ind, A_val = [], []
    for j in range(n):
        for i, v in sorted(entries[j]):
            A_ind.append(i)
            A_val.append(v)
        A_ptr[j + 1] = len(A_ind)
    return Problem(m=m, n=n, dir=direction, c0=0.0,
                   row_type=_i8(rtype), row_lb=_f8(rlb), row_ub=_f8(rub), rii=np.ones(m),
                   row_stat=_i8(np.full(m, GLP_BS)), col_type=_i8(ctype), col_lb=_f8(clb), col_ub=_f8(cub),
                   col_coef=_f8([obj.get(j, 0.0) for j in range(n)]), sjj=np.ones(n), col_stat=_i8(cstat),
                   col_kind=_i8([GLP_IV if j in isint else GLP_CV for j in range(n)]), A_ptr=A_ptr,
                   A_ind=_i4(A_ind), A_val=_f8(A_val), name="")


# ---------------------------------------------------------------------------
# MPS reader (fixed or free format; SURVEY.md §8(f): the configs' netlib
# 25fv47 and MIPLIB mas76 are MPS files, which the reference cannot read).
# Conventions of GLPK's glp_read_mps (glpmps.c, GLPK 4.49): rows in ROWS
# order (the first N row is the objective, other N rows are dropped), columns
# in COLUMNS order, RHS on the objective row = minus the constant term, RANGES
# per row type, BOUNDS types UP/LO/FX/FR/MI/PL/BV/LI/UI (UP with a negative
# value and no lower bound makes the lower bound -inf), integer columns from
# MARKER INTORG / INTEND keep the default bounds [0, +inf); column lists
# sorted by row.  Parity is by content: the same LP written in CPLEX LP form
# reads to the same problem (tests/test_readers.py).
# ---------------------------------------------------------------------------
class MpsFormatError(ValueError):
    pass


def read_mps(text: str, free: bool = True) -> Problem:
    BIG = 1.7976931348623157e308
    section = None
    rows: dict[str, int] = {}
    row_names: list[str] = []
    row_kind: list[str] = []
    obj_name = None
    cols: dict[str, int] = {}
    col_int: list[bool] = []
    entries: list[list[tuple[int, float]]] = []
    coef: list[float] = []
    rhs: dict[int, float] = {}
    rng: dict[int, float] = {}
    lbs: list[float] = []
    ubs: list[float] = []
    seen_lb: list[bool] = []
    seen_ub: list[bool] = []
    c0 = 0.0
    in_int = False
    direction = GLP_MIN

    def fields(line: str) -> list[str]:
        if free:
            return line.split()
        # fixed MPS: columns 2-3, 5-12, 15-22, 25-36, 40-47, 50-61
        spans = ((1, 3), (4, 12), (14, 22), (24, 36), (39, 47), (49, 61))
        out = [line[a:b].strip() for a, b in spans]
        while out and out[-1] == "":
            out.pop()
        if out and out[0] == "" and section not in ("ROWS", "BOUNDS"):
            out.pop(0)          # the blank type field of COLUMNS/RHS/RANGES
        return out

    for ln, raw in enumerate(text.splitlines(), 1):
        if not raw.strip() or raw.startswith("*"):
            continue
        if not raw[0].isspace():
            head = raw.split()
            section = head[0].upper()
            if section == "OBJSENSE" and len(head) > 1:
                direction = GLP_MAX if head[1].upper().startswith("MAX") else GLP_MIN
            if section == "ENDATA":
                break
            continue
        f = fields(raw)
        if section == "OBJSENSE":
            direction = GLP_MAX if f[0].upper().startswith("MAX") else GLP_MIN
        elif section == "ROWS":
            kind, name = f[0].upper(), f[1]
            if kind == "N":
                if obj_name is None:
                    obj_name = name
                continue
            if kind not in ("L", "G", "E"):
                raise MpsFormatError(f"{ln}: row type `{kind}' not recognized")
            rows[name] = len(row_names)
            row_names.append(name)
            row_kind.append(kind)
        elif section == "COLUMNS":
            if len(f) >= 3 and f[1].upper() == "'MARKER'":
                tag = f[-1].upper()
                in_int = tag == "'INTORG'"
                continue
            name = f[0]
            if name not in cols:
                cols[name] = len(entries)
                entries.append([])
                coef.append(0.0)
                col_int.append(in_int)
                lbs.append(0.0); ubs.append(+BIG); seen_lb.append(False); seen_ub.append(False)
            j = cols[name]
            for k in range(1, len(f) - 1, 2):
                rname, v = f[k], float(f[k + 1])
                if rname == obj_name:
                    coef[j] = v
                elif rname in rows:
                    if v != 0.0:
                        entries[j].append((rows[rname] + 1, v))
                else:
                    raise MpsFormatError(f"{ln}: row `{rname}' not found")
        elif section in ("RHS", "RANGES"):
            start = 1 if len(f) % 2 == 1 else 0
            for k in range(start, len(f) - 1, 2):
                rname, v = f[k], float(f[k + 1])
                if rname == obj_name and section == "RHS":
                    c0 = -v
                elif rname in rows:
                    (rhs if section == "RHS" else rng)[rows[rname]] = v
                else:
                    raise MpsFormatError(f"{ln}: row `{rname}' not found")
        elif section == "BOUNDS":
            kind = f[0].upper()
            name = f[2] if len(f) >= 3 else f[1]
            v = float(f[3]) if len(f) >= 4 else 0.0
            if name not in cols:
                raise MpsFormatError(f"{ln}: column `{name}' not found")
            j = cols[name]
            if kind == "UP":
                ubs[j] = v
                if v < 0.0 and not seen_lb[j]:
                    lbs[j] = -BIG
                seen_ub[j] = True
            elif kind in ("LO", "LI"):
                lbs[j] = v
                seen_lb[j] = True
                if kind == "LI":
                    col_int[j] = True
            elif kind == "UI":
                ubs[j] = v
                col_int[j] = True
                seen_ub[j] = True
            elif kind == "FX":
                lbs[j] = ubs[j] = v
                seen_lb[j] = seen_ub[j] = True
            elif kind == "FR":
                lbs[j], ubs[j] = -BIG, +BIG
            elif kind == "MI":
                lbs[j] = -BIG
            elif kind == "PL":
                ubs[j] = +BIG
            elif kind == "BV":
                lbs[j], ubs[j] = 0.0, 1.0
                col_int[j] = True
            else:
                raise MpsFormatError(f"{ln}: bound type `{kind}' not recognized")
        elif section in ("NAME",):
            continue
        else:
            raise MpsFormatError(f"{ln}: data line outside a known section")
    m, n = len(row_names), len(entries)
    rtype, rlb, rub = [], [], []
    for i in range(m):
        b = rhs.get(i, 0.0)
        kind = row_kind[i]
        if i in rng:
            r = rng[i]
            if kind == "E":
                lo, hi = (b, b + abs(r)) if r >= 0.0 else (b - abs(r), b)
            elif kind == "L":
                lo, hi = b - abs(r), b
            else:
                lo, hi = b, b + abs(r)
            t = GLP_FX if lo == hi else GLP_DB
        elif kind == "L":
            t, lo, hi = GLP_UP, 0.0, b
        elif kind == "G":
            t, lo, hi = GLP_LO, b, 0.0
        else:
            t, lo, hi = GLP_FX, b, b
        rtype.append(t); rlb.append(lo); rub.append(hi)
    ctype, clb, cub, cstat = [], [], [], []
    for j in range(n):
        lb, ub = lbs[j], ubs[j]
        if lb == -BIG and ub == +BIG:
            t, l, u, st = GLP_FR, 0.0, 0.0, GLP_NF
        elif ub == +BIG:
            t, l, u, st = GLP_LO, lb, 0.0, GLP_NL
        elif lb == -BIG:
            t, l, u, st = GLP_UP, 0.0, ub, GLP_NU
        elif lb != ub:
            t, l, u, st = GLP_DB, lb, ub, GLP_NL
        else:
            t, l, u, st = GLP_FX, lb, ub, GLP_NS
        ctype.append(t); clb.append(l); cub.append(u); cstat.append(st)
    A_ptr = np.zeros(n + 1, np.int32)
    A_ind, A_val = [], []
    for j in range(n):
        for i, v in sorted(entries[j]):
            A_ind.append(i)
            A_val.append(v)
        A_ptr[j + 1] = len(A_ind)
    return Problem(m=m, n=n, dir=direction, c0=c0,
                   row_type=_i8(rtype), row_lb=_f8(rlb), row_ub=_f8(rub), rii=np.ones(m),
                   row_stat=_i8(np.full(m, GLP_BS)), col_type=_i8(ctype), col_lb=_f8(clb), col_ub=_f8(cub),
                   col_coef=_f8(coef), sjj=np.ones(n), col_stat=_i8(cstat),
                   col_kind=_i8([GLP_IV if t else GLP_CV for t in col_int]), A_ptr=A_ptr,
                   A_ind=_i4(A_ind), A_val=_f8(A_val), name="")


def write_mps(p: Problem) -> str:
    """Free MPS text of a Problem (the inverse of read_mps, unscaled data)."""
    def _num(v) -> str:
        return repr(float(v))

    out = ["NAME " + (p.name or "problem")]
    if p.dir == GLP_MAX:
        out += ["OBJSENSE", "    MAX"]
    out += ["ROWS", " N obj"]
    kind = {GLP_UP: "L", GLP_LO: "G", GLP_FX: "E", GLP_DB: "L", GLP_FR: "N"}
    for i in range(p.m):
        if p.row_type[i] == GLP_FR:
            raise ValueError("free rows are not written")
        out.append(f" {kind[int(p.row_type[i])]} r{i + 1}")
    out.append("COLUMNS")
    in_int = False
    for j in range(p.n):
        isint = p.col_kind[j] == GLP_IV
        if isint != in_int:
            out.append("    MARKER 'MARKER' " + ("'INTORG'" if isint else "'INTEND'"))
            in_int = isint
        if p.col_coef[j] != 0.0:
            out.append(f"    c{j + 1} obj {_num(p.col_coef[j])}")
        for t in range(p.A_ptr[j], p.A_ptr[j + 1]):
            out.append(f"    c{j + 1} r{p.A_ind[t]} {_num(p.A_val[t])}")
    if in_int:
        out.append("    MARKER 'MARKER' 'INTEND'")
    out.append("RHS")
    if p.c0 != 0.0:
        out.append(f"    RHS obj {_num(-p.c0)}")
    for i in range(p.m):
        t = int(p.row_type[i])
        b = p.row_ub[i] if t in (GLP_UP, GLP_DB) else p.row_lb[i]
        if b != 0.0:
            out.append(f"    RHS r{i + 1} {_num(b)}")
    rng = [f"    RNG r{i + 1} {_num(p.row_ub[i] - p.row_lb[i])}" for i in range(p.m) if p.row_type[i] == GLP_DB]
    if rng:
        out += ["RANGES"] + rng
    out.append("BOUNDS")
    for j in range(p.n):
        t, lb, ub = int(p.col_type[j]), p.col_lb[j], p.col_ub[j]
        c = f"c{j + 1}"
        if t == GLP_FR:
            out.append(f" FR BND {c}")
        elif t == GLP_LO:
            if lb != 0.0:
                out.append(f" LO BND {c} {_num(lb)}")
        elif t == GLP_UP:
            out += [f" MI BND {c}", f" UP BND {c} {_num(ub)}"]
        elif t == GLP_DB:
            out += [f" LO BND {c} {_num(lb)}", f" UP BND {c} {_num(ub)}"]
        else:
            out.append(f" FX BND {c} {_num(lb)}")
    out.append("ENDATA")
    return "\n".join(out) + "\n"
