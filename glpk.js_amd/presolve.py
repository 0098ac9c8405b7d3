"""The presolve paths of glp_simplex and glp_intopt (presolve = GLP_ON) on the
Python host: preprocess_and_solve_lp (glpapi06.js:41-147) and
preprocess_and_solve_mip (glpapi09.js:116-250).

The preprocessor itself is native (gk_npp_*, glpk.js_amd/csrc/gk_npp.cc, a
restatement of glpnpp01.js .. glpnpp05.js); the reduced problem is scaled
(gk_scale_prob), given the triangular starting basis (gk_adv_basis) and
solved by the device simplex / branch-and-bound like any other problem, then
its solution is carried back through the transformation stack."""
from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np

from . import gk
from .problems import (GLP_BS, GLP_DB, GLP_FEAS, GLP_NOFEAS, GLP_UNBND, Problem,
                       _col_stat_for)

GLP_SOL, GLP_MIP = 1, 3
GLP_MSG_ERR, GLP_MSG_ON, GLP_MSG_ALL = 1, 2, 3


def _bind(L):
    if getattr(L, "_npp_bound", False):
        return L
    P = C.c_void_p
    L.gk_npp_create.restype = P
    L.gk_npp_create.argtypes = []
    L.gk_npp_destroy.argtypes = [P]
    L.gk_npp_destroy.restype = None
    L.gk_npp_load.argtypes = [P, P, P, C.c_int]
    L.gk_npp_simplex.argtypes = [P]
    L.gk_npp_integer.argtypes = [P, C.c_int, P]
    L.gk_npp_build_size.argtypes = [P, P, P, P]
    L.gk_npp_build.argtypes = [P] + [P] * 14
    L.gk_npp_postprocess.argtypes = [P, C.c_int, C.c_int, P, P, P, P]
    L.gk_npp_unload_sol.argtypes = [P, P]
    L.gk_npp_unload_mip.argtypes = [P, P, P, P, P, P, P]
    for f in ("gk_npp_load", "gk_npp_simplex", "gk_npp_integer", "gk_npp_build_size", "gk_npp_build",
              "gk_npp_postprocess", "gk_npp_unload_sol", "gk_npp_unload_mip"):
        getattr(L, f).restype = C.c_int
    L._npp_bound = True
    return L


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class Npp:
    """One preprocessor workspace (npp_create_wksp .. npp_unload_sol)."""

    def __init__(self, L=None):
        self.L = _bind(L or gk.load_library())
        self.h = self.L.gk_npp_create()
        if not self.h:
            raise gk.GkError(gk._err(self.L))
        self.row_ref = self.col_ref = None

    def __del__(self):
        if getattr(self, "h", None):
            self.L.gk_npp_destroy(self.h)
            self.h = None

    def _check(self, ret):
        if ret == gk.GK_EABI:
            raise gk.GkError(gk._err(self.L))
        return ret

    def load(self, lp: gk.Lp, col_kind: np.ndarray | None, sol: int):
        """npp_load_prob (glpnpp01.js:262); lp: the original problem's gk_lp
        (its arrays must stay alive), col_kind [0..n] for GLP_MIP."""
        self._lp = lp
        self._kind = None if col_kind is None else np.ascontiguousarray(col_kind, np.int8)
        self._check(self.L.gk_npp_load(self.h, C.byref(lp), _ptr(self._kind), sol))

    def simplex(self) -> int:
        return self._check(self.L.gk_npp_simplex(self.h))

    def integer(self, binarize: bool) -> tuple[int, list]:
        msg = np.zeros(7, np.int32)
        ret = self._check(self.L.gk_npp_integer(self.h, 1 if binarize else 0, _ptr(msg)))
        return ret, msg.tolist()

    def build(self, dir_: int) -> Problem:
        """npp_build_prob (glpnpp01.js:396): the reduced problem."""
        m, n, nnz = C.c_int(), C.c_int(), C.c_int()
        self._check(self.L.gk_npp_build_size(self.h, C.byref(m), C.byref(n), C.byref(nnz)))
        m, n, nnz = m.value, n.value, nnz.value
        rt, rl, ru = np.zeros(m + 1, np.int8), np.zeros(m + 1), np.zeros(m + 1)
        ct, cl, cu, cc = np.zeros(n + 1, np.int8), np.zeros(n + 1), np.zeros(n + 1), np.zeros(n + 1)
        ck = np.zeros(n + 1, np.int8)
        ap, ai, av = np.zeros(n + 2, np.int32), np.zeros(nnz + 1, np.int32), np.zeros(nnz + 1)
        rr, cr = np.zeros(m + 1, np.int32), np.zeros(n + 1, np.int32)
        c0 = C.c_double()
        self._check(self.L.gk_npp_build(self.h, _ptr(rt), _ptr(rl), _ptr(ru), _ptr(ct), _ptr(cl), _ptr(cu),
                                        _ptr(cc), _ptr(ck), _ptr(ap), _ptr(ai), _ptr(av), _ptr(rr), _ptr(cr),
                                        C.byref(c0)))
        self.row_ref, self.col_ref = rr[1:].copy(), cr[1:].copy()
        A_ptr = (ap[1:] - 1).astype(np.int32) if n > 0 else np.zeros(1, np.int32)
        return Problem(m=m, n=n, dir=dir_, c0=c0.value, row_type=rt[1:].copy(), row_lb=rl[1:].copy(),
                       row_ub=ru[1:].copy(), rii=np.ones(m), row_stat=np.full(m, GLP_BS, np.int8),
                       col_type=ct[1:].copy(), col_lb=cl[1:].copy(), col_ub=cu[1:].copy(),
                       col_coef=cc[1:].copy(), sjj=np.ones(n),
                       col_stat=_col_stat_for(ct[1:], cl[1:], cu[1:]), col_kind=ck[1:].copy(),
                       A_ptr=A_ptr, A_ind=ai[1:].copy(), A_val=av[1:].copy(), name="presolved")

    def postprocess_sol(self, pbs, dbs, row_stat, row_dual, col_stat, col_prim):
        """npp_postprocess for a basic solution; arrays [0..m] / [0..n]."""
        a = [np.ascontiguousarray(x, t) for x, t in ((row_stat, np.int8), (row_dual, np.float64),
                                                      (col_stat, np.int8), (col_prim, np.float64))]
        self._check(self.L.gk_npp_postprocess(self.h, pbs, dbs, *[_ptr(x) for x in a]))

    def postprocess_mip(self, mip_stat, col_mipx):
        x = np.ascontiguousarray(col_mipx, np.float64)
        self._check(self.L.gk_npp_postprocess(self.h, mip_stat, 0, None, None, None, _ptr(x)))

    def unload_sol(self, P: gk.GkProblem):
        """npp_unload_sol (glpnpp01.js:572) into P (statuses, values, objective)."""
        lp = P._lp_struct()
        self._check(self.L.gk_npp_unload_sol(self.h, C.byref(lp)))
        P.pbs_stat, P.dbs_stat, P.obj_val, P.some, P.valid = lp.pbs_stat, lp.dbs_stat, lp.obj_val, 0, 0

    def unload_mip(self, P: gk.GkProblem) -> None:
        lp = P._lp_struct()
        st, obj = C.c_int(), C.c_double()
        self._check(self.L.gk_npp_unload_mip(self.h, C.byref(lp), _ptr(P.col_kind), _ptr(P.row_mipx),
                                             _ptr(P.col_mipx), C.byref(st), C.byref(obj)))
        P.mip_stat, P.mip_obj = st.value, obj.value


def problem_lp(p: Problem) -> tuple:
    """A gk_lp over a problems.Problem with solution arrays of its own, for
    the host-only steps (load, unload) without a device: (lp, arrays)."""
    m, n = p.m, p.n
    pad = gk._pad
    a = dict(row_type=pad(p.row_type, np.int8), row_lb=pad(p.row_lb, np.float64), row_ub=pad(p.row_ub, np.float64),
             rii=pad(p.rii, np.float64), col_type=pad(p.col_type, np.int8), col_lb=pad(p.col_lb, np.float64),
             col_ub=pad(p.col_ub, np.float64), col_coef=pad(p.col_coef, np.float64), sjj=pad(p.sjj, np.float64),
             A_ptr=pad(np.asarray(p.A_ptr, np.int32) + 1, np.int32), A_ind=pad(p.A_ind, np.int32),
             A_val=pad(p.A_val, np.float64), head=np.zeros(m + 1, np.int32),
             row_stat=pad(p.row_stat, np.int8), col_stat=pad(p.col_stat, np.int8),
             row_bind=np.zeros(m + 1, np.int32), col_bind=np.zeros(n + 1, np.int32),
             row_prim=np.zeros(m + 1), row_dual=np.zeros(m + 1), col_prim=np.zeros(n + 1), col_dual=np.zeros(n + 1),
             col_kind=pad(p.col_kind, np.int8), row_mipx=np.zeros(m + 1), col_mipx=np.zeros(n + 1))
    lp = gk.Lp()
    lp.m, lp.n, lp.nnz, lp.dir, lp.c0 = m, n, p.nnz, p.dir, p.c0
    for k in ("row_type", "row_lb", "row_ub", "rii", "col_type", "col_lb", "col_ub", "col_coef", "sjj", "A_ptr",
              "A_ind", "A_val", "head", "row_stat", "col_stat", "row_bind", "col_bind", "row_prim", "row_dual",
              "col_prim", "col_dual"):
        setattr(lp, k, _ptr(a[k]))
    return lp, a


@contextlib.contextmanager
def _term_out(on: bool):
    """env.term_out around a nested routine (glpapi06.js:109-116)."""
    if on:
        yield
        return
    keep = gk._print_func
    gk.glp_set_print_func(lambda s: None)
    try:
        yield
    finally:
        gk.glp_set_print_func(keep)


def _reduced(P: gk.GkProblem, red: Problem) -> gk.GkProblem:
    lp = gk.GkProblem(P.ctx, red)
    if P.bfcp is not None:
        lp.set_bfcp(**{k: getattr(P.bfcp, k) for k, _ in gk.Bfcp._fields_})
    return lp


def preprocess_and_solve_lp(P: gk.GkProblem, parm) -> int:
    """glpapi06.js:41-147."""
    out = gk._xprintf
    if parm.msg_lev >= GLP_MSG_ALL:
        out("Preprocessing...")
    npp = Npp(P.L)
    npp.load(P._lp_struct(), None, GLP_SOL)
    ret = npp.simplex()
    if ret == gk.GLP_ENOPFS:
        if parm.msg_lev >= GLP_MSG_ALL:
            out("PROBLEM HAS NO PRIMAL FEASIBLE SOLUTION")
    elif ret == gk.GLP_ENODFS:
        if parm.msg_lev >= GLP_MSG_ALL:
            out("PROBLEM HAS NO DUAL FEASIBLE SOLUTION")
    if ret != 0:
        return ret
    red = npp.build(P.dir)
    if red.m == 0 and red.n == 0:
        # the empty reduced LP has the empty optimal solution
        if parm.msg_lev >= GLP_MSG_ON and parm.out_dly == 0:
            out(f"{P.it_cnt}: obj = {gk._js_num(red.c0)}  infeas = 0.0")
        if parm.msg_lev >= GLP_MSG_ALL:
            out("OPTIMAL SOLUTION FOUND BY LP PREPROCESSOR")
        e8, ef = np.zeros(1, np.int8), np.zeros(1)
        npp.postprocess_sol(GLP_FEAS, GLP_FEAS, e8, ef, e8, ef)
        npp.unload_sol(P)
        return 0
    if parm.msg_lev >= GLP_MSG_ALL:
        out(f"{red.m} row{'' if red.m == 1 else 's'}, {red.n} column{'' if red.n == 1 else 's'}, "
            f"{red.nnz} non-zero{'' if red.nnz == 1 else 's'}")
    lp = _reduced(P, red)
    with _term_out(parm.msg_lev >= GLP_MSG_ALL):
        gk.glp_scale_prob(lp, gk.GLP_SF_AUTO)
    with _term_out(parm.msg_lev >= GLP_MSG_ALL):
        gk.glp_adv_basis(lp, 0)
    lp.it_cnt = P.it_cnt
    ret = gk._solve_lp(lp, parm)
    P.it_cnt = lp.it_cnt
    if not (ret == 0 and lp.pbs_stat == GLP_FEAS and lp.dbs_stat == GLP_FEAS):
        if parm.msg_lev >= GLP_MSG_ERR:
            out("glp_simplex: unable to recover undefined or non-optimal solution")
        if ret == 0:
            if lp.pbs_stat == GLP_NOFEAS:
                ret = gk.GLP_ENOPFS
            elif lp.dbs_stat == GLP_NOFEAS:
                ret = gk.GLP_ENODFS
            else:
                raise gk.GkError("glp_simplex: reduced problem left without a status")
        return ret
    npp.postprocess_sol(lp.pbs_stat, lp.dbs_stat, lp.row_stat, lp.row_dual, lp.col_stat, lp.col_prim)
    npp.unload_sol(P)
    return 0


def _lp_status(lp: gk.GkProblem) -> int:
    """glp_get_status (glpapi02.js) of a basic solution."""
    st = lp.pbs_stat
    if st == GLP_FEAS:
        if lp.dbs_stat == GLP_NOFEAS:
            st = GLP_UNBND
        elif lp.dbs_stat == GLP_FEAS:
            st = gk.GLP_OPT
    return st


def preprocess_and_solve_mip(P: gk.GkProblem, parm, binarize: bool = False) -> int:
    """glpapi09.js:116-250."""
    out = gk._xprintf
    all_ = parm.msg_lev >= GLP_MSG_ALL
    if all_:
        out("Preprocessing...")
    npp = Npp(P.L)
    npp.load(P._lp_struct(), P.col_kind, GLP_MIP)
    ret, msg = npp.integer(binarize)
    if all_ and ret == 0:
        # npp_integer's own lines (glpnpp04.js:92-97, glpnpp05.js:475-514)
        if msg[0] > 0:
            out(f"{msg[0]} integer variable(s) were replaced by {msg[1]} binary ones")
        if msg[2] > 0:
            out(f"{msg[2]} row(s) were added due to binarization")
        if msg[3] > 0:
            out(f"Binarization failed for {msg[3]} integer variable(s)")
        if msg[4] > 0:
            out(f"{msg[4]} hidden packing inequaliti(es) were detected")
        if msg[5] > 0:
            out(f"{msg[5]} hidden covering inequaliti(es) were detected")
        if msg[6] > 0:
            out(f"{msg[6]} constraint coefficient(s) were reduced")
    if ret == gk.GLP_ENOPFS:
        if all_:
            out("PROBLEM HAS NO PRIMAL FEASIBLE SOLUTION")
    elif ret == gk.GLP_ENODFS:
        if all_:
            out("LP RELAXATION HAS NO DUAL FEASIBLE SOLUTION")
    if ret != 0:
        return ret
    red = npp.build(P.dir)
    if red.m == 0 and red.n == 0:
        if all_:
            out(f"Objective value = {gk._js_num(red.c0)}")
            out("INTEGER OPTIMAL SOLUTION FOUND BY MIP PREPROCESSOR")
        npp.postprocess_mip(gk.GLP_OPT, np.zeros(1))
        npp.unload_mip(P)
        return 0
    if all_:
        iv = red.col_kind == gk.GLP_IV
        ni = int(np.count_nonzero(iv))
        nb = int(np.count_nonzero(iv & (red.col_type == GLP_DB) & (red.col_lb == 0.0) & (red.col_ub == 1.0)))
        s = ("none of" if nb == 0 else "" if (ni == 1 and nb == 1) else "one of" if nb == 1 else
             "all of" if nb == ni else f"{nb} of")
        out(f"{red.m} row{'' if red.m == 1 else 's'}, {red.n} column{'' if red.n == 1 else 's'}, "
            f"{red.nnz} non-zero{'' if red.nnz == 1 else 's'}")
        out(f"{ni} integer variable{'' if ni == 1 else 's'}, {s} which {'is' if nb == 1 else 'are'} binary")
    mip = _reduced(P, red)
    with _term_out(all_):
        gk.glp_scale_prob(mip, gk.GLP_SF_GM | gk.GLP_SF_EQ | gk.GLP_SF_2N | gk.GLP_SF_SKIP)
    with _term_out(all_):
        gk.glp_adv_basis(mip, 0)
    if all_:
        out("Solving LP relaxation...")
    mip.it_cnt = P.it_cnt
    ret = gk.glp_simplex(mip, gk.SMCP(msg_lev=parm.msg_lev))
    P.it_cnt = mip.it_cnt
    if ret != 0:
        if parm.msg_lev >= GLP_MSG_ERR:
            out("glp_intopt: cannot solve LP relaxation")
        return gk.GLP_EFAIL
    st = _lp_status(mip)
    if st == gk.GLP_OPT:
        ret = 0
    elif st == GLP_NOFEAS:
        ret = gk.GLP_ENOPFS
    elif st == GLP_UNBND:
        ret = gk.GLP_ENODFS
    else:
        raise gk.GkError(f"glp_intopt: LP relaxation status {st}")
    if ret != 0:
        return ret
    mip.it_cnt = P.it_cnt
    ret = gk._solve_mip(mip, parm, None, 0)
    P.it_cnt = mip.it_cnt
    P.mip_stats = mip.mip_stats
    if not (mip.mip_stat == gk.GLP_OPT or mip.mip_stat == GLP_FEAS):
        P.mip_stat = mip.mip_stat
        return ret
    npp.postprocess_mip(mip.mip_stat, mip.col_mipx)
    npp.unload_mip(P)
    return ret
