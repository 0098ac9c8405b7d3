"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/_build/liboracle.so, the bit-faithful C restatement of
the reference's simplex / branch-and-bound path.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module;
the product path (glpk.js_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_TRACE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                        C.c_int, C.c_double)


class SmcpFlat(C.Structure):
    """0 / 0.0 fields keep the SMCP default, like SMCP's `options[x] || default`."""
    _fields_ = [("meth", C.c_int), ("pricing", C.c_int), ("r_test", C.c_int), ("it_lim", C.c_int),
                ("tm_lim", C.c_int), ("tol_bnd", C.c_double), ("tol_dj", C.c_double),
                ("tol_piv", C.c_double), ("obj_ll", C.c_double), ("obj_ul", C.c_double)]


class IocpFlat(C.Structure):
    _fields_ = [("br_tech", C.c_int), ("bt_tech", C.c_int), ("pp_tech", C.c_int), ("tm_lim", C.c_int),
                ("tol_int", C.c_double), ("tol_obj", C.c_double), ("mip_gap", C.c_double)]


class ResultFlat(C.Structure):
    _fields_ = [("pbs_stat", C.c_int), ("dbs_stat", C.c_int), ("some", C.c_int), ("it_cnt", C.c_int),
                ("valid", C.c_int), ("mip_stat", C.c_int), ("obj_val", C.c_double), ("mip_obj", C.c_double)]


class IosStats(C.Structure):
    _fields_ = [("lp_solves", C.c_long), ("nodes_created", C.c_long), ("node_visits", C.c_long),
                ("pivots", C.c_long)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        i8p = np.ctypeslib.ndpointer(np.int8, flags="C")
        f8p = np.ctypeslib.ndpointer(np.float64, flags="C")
        i4p = np.ctypeslib.ndpointer(np.int32, flags="C")
        L.orc_prob_create.restype = P
        L.orc_prob_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double,
                                      i8p, f8p, f8p, f8p, i8p,
                                      i8p, f8p, f8p, f8p, f8p, i8p, i8p,
                                      i4p, i4p, f8p]
        L.orc_prob_delete.argtypes = [P]
        L.orc_prob_simplex.argtypes = [P, C.POINTER(SmcpFlat), _TRACE_FN, P]
        L.orc_prob_simplex.restype = C.c_int
        L.orc_prob_result.argtypes = [P, C.POINTER(ResultFlat)] + [C.c_void_p] * 9
        L.orc_prob_factorize.argtypes = [P]
        L.orc_prob_ftran.argtypes = [P, f8p, C.c_int]
        L.orc_prob_set_bfcp.argtypes = [P, C.c_int, C.c_int, C.c_int]
        L.orc_prob_set_upd_tol.argtypes = [P, C.c_double]
        L.orc_set_lpf_fix.argtypes = [C.c_int]
        L.orc_last_error.restype = C.c_char_p
        L.orc_scale_prob.argtypes = [C.c_int, C.c_int, i4p, i4p, f8p, C.c_int, f8p, f8p, f8p]
        L.orc_scale_prob.restype = C.c_int
        L.orc_instab_count.restype = C.c_long
        L.orc_instab_count.argtypes = [C.POINTER(C.c_int)]
        if hasattr(L, "orc_prob_intopt"):
            L.orc_prob_intopt.argtypes = [P, C.POINTER(IocpFlat), C.POINTER(IosStats)]
            L.orc_prob_intopt.restype = C.c_int
        _lib = L
    return _lib


class OracleError(RuntimeError):
    pass


class OracleProb:
    """The reference problem object restricted to the hot path, in C."""

    def __init__(self, p):
        L = lib()
        self.m, self.n = p.m, p.n
        self._keep = p
        self.h = L.orc_prob_create(p.m, p.n, p.dir, p.c0, p.row_type, p.row_lb, p.row_ub, p.rii,
                                   p.row_stat, p.col_type, p.col_lb, p.col_ub, p.col_coef, p.sjj,
                                   p.col_stat, p.col_kind, p.A_ptr, p.A_ind, p.A_val)
        if not self.h:
            raise OracleError(L.orc_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_prob_delete(self.h)
            self.h = None

    def set_bfcp(self, type_, nfs_max=0, nrs_max=0, upd_tol=None):
        lib().orc_prob_set_bfcp(self.h, type_, nfs_max, nrs_max)
        if upd_tol is not None:
            lib().orc_prob_set_upd_tol(self.h, upd_tol)

    def simplex(self, trace: list | None = None, **opts) -> int:
        f = SmcpFlat(**{k: v for k, v in opts.items() if k in dict(SmcpFlat._fields_)})
        if trace is not None:
            def cb(_ctx, kind, it, phase, p, q, kq, kp, t):
                trace.append((it, phase, p, q, kq, kp, t))
            fn = _TRACE_FN(cb)
        else:
            fn = _TRACE_FN()
        ret = lib().orc_prob_simplex(self.h, C.byref(f), fn, None)
        if ret < 0:
            raise OracleError(lib().orc_last_error().decode())
        return ret

    def intopt(self, **opts):
        f = IocpFlat(**{k: v for k, v in opts.items() if k in dict(IocpFlat._fields_)})
        st = IosStats()
        ret = lib().orc_prob_intopt(self.h, C.byref(f), C.byref(st))
        if ret < 0:
            raise OracleError(lib().orc_last_error().decode())
        return ret, st

    def factorize(self) -> int:
        return lib().orc_prob_factorize(self.h)

    def ftran(self, x: np.ndarray, tr: bool = False) -> np.ndarray:
        y = np.ascontiguousarray(x, dtype=np.float64).copy()
        if lib().orc_prob_ftran(self.h, y, 1 if tr else 0) < 0:
            raise OracleError(lib().orc_last_error().decode())
        return y

    def result(self) -> dict:
        m, n = self.m, self.n
        r = ResultFlat()
        a = {"row_stat": np.zeros(m, np.int8), "row_prim": np.zeros(m), "row_dual": np.zeros(m),
             "col_stat": np.zeros(n, np.int8), "col_prim": np.zeros(n), "col_dual": np.zeros(n),
             "row_mipx": np.zeros(m), "col_mipx": np.zeros(n), "head": np.zeros(m, np.int32)}
        ptr = lambda v: v.ctypes.data_as(C.c_void_p)
        lib().orc_prob_result(self.h, C.byref(r), ptr(a["row_stat"]), ptr(a["row_prim"]), ptr(a["row_dual"]),
                              ptr(a["col_stat"]), ptr(a["col_prim"]), ptr(a["col_dual"]),
                              ptr(a["row_mipx"]), ptr(a["col_mipx"]), ptr(a["head"]))
        out = {k: getattr(r, k) for k, _ in ResultFlat._fields_}
        out.update(a)
        return out


def set_lpf_fix(on: bool):
    """Schur-complement update with the C original's offsets (oracle/lpf.c)
    instead of glplpf.js:420/:422's idx 0."""
    lib().orc_set_lpf_fix(1 if on else 0)


def instab_count():
    """(number of "numerical instability" restarts so far, it_cnt of the last)"""
    it = C.c_int(-1)
    n = lib().orc_instab_count(C.byref(it))
    return n, it.value


def scale_prob(m: int, n: int, A_ptr, A_ind, A_val, flags: int):
    """glp_scale_prob restated (oracle/scale.c): (ret, rii[m], sjj[n],
    report[13]) for the CSC matrix (0-based offsets, 1-based rows)."""
    rii, sjj, rep = np.ones(max(m, 1)), np.ones(max(n, 1)), np.zeros(13)
    ret = lib().orc_scale_prob(m, n, np.ascontiguousarray(A_ptr, np.int32), np.ascontiguousarray(A_ind, np.int32),
                               np.ascontiguousarray(A_val, np.float64), int(flags), rii, sjj, rep)
    return ret, rii[:m], sjj[:n], rep
