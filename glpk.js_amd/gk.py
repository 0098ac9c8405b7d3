"""Host-side mirror of the reference interface for the hot path, over the C-ABI.

`glp_simplex(P, SMCP(...))` and `glp_factorize(P)` follow glpapi06.js:1-340
and glpapi12.js:5-100 (parameter checks, the double-bound check, the trivial
LP for nnz == 0, solve_lp's factorize-then-spx flow, GLP_DUALP's fallback to
the primal), with spx_primal / spx_dual / bfd_* executed by
libglpk_mi355x.so on the MI355X.  There is no CPU fallback: if the library
or a gfx950 device is missing, `Context()` raises.

Arrays crossing the boundary are 1-based like the reference's typed arrays
(element 0 unused); `Problem` (problems.py) holds them 0-based and this
module pads them.
"""
from __future__ import annotations

import ctypes as C
import operator
import os

import numpy as np

from .problems import (GLP_BS, GLP_DB, GLP_DUAL, GLP_DUALP, GLP_FEAS, GLP_FX, GLP_LO, GLP_MAX, GLP_MIN,
                       GLP_NF, GLP_NL, GLP_NOFEAS, GLP_NS, GLP_NU, GLP_PRIMAL, GLP_UNDEF, GLP_UP, GLP_FR,
                       GLP_ETMLIM, Problem)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libglpk_mi355x.so")

GLP_MSG_OFF, GLP_MSG_ERR, GLP_MSG_ON, GLP_MSG_ALL, GLP_MSG_DBG = 0, 1, 2, 3, 4
GLP_VERSION = "4.49"                         # glp_version (glpapi.js:76, glpk.js:3-4)
GLP_PT_STD, GLP_PT_PSE = 0x11, 0x22
GLP_RT_STD, GLP_RT_HAR = 0x11, 0x22
GLP_EBADB, GLP_ESING, GLP_ECOND, GLP_EBOUND, GLP_EFAIL = 1, 2, 3, 4, 5
INT_MAX = 0x7FFFFFFF
DBL_MAX = np.finfo(np.float64).max
GK_EABI = -1


class GkError(RuntimeError):
    """Contract violation reported by the C-ABI (the reference's xerror)."""


class Bfcp(C.Structure):
    _fields_ = [("type", C.c_int), ("lu_size", C.c_int), ("piv_tol", C.c_double), ("piv_lim", C.c_int),
                ("suhl", C.c_int), ("eps_tol", C.c_double), ("max_gro", C.c_double), ("nfs_max", C.c_int),
                ("upd_tol", C.c_double), ("nrs_max", C.c_int), ("rs_size", C.c_int)]


class Smcp(C.Structure):
    _fields_ = [("msg_lev", C.c_int), ("meth", C.c_int), ("pricing", C.c_int), ("r_test", C.c_int),
                ("tol_bnd", C.c_double), ("tol_dj", C.c_double), ("tol_piv", C.c_double),
                ("obj_ll", C.c_double), ("obj_ul", C.c_double),
                ("it_lim", C.c_int), ("tm_lim", C.c_int), ("out_frq", C.c_int), ("out_dly", C.c_int),
                ("presolve", C.c_int)]


class Lp(C.Structure):
    _fields_ = [("m", C.c_int), ("n", C.c_int), ("nnz", C.c_int), ("dir", C.c_int), ("c0", C.c_double),
                ("row_type", C.c_void_p), ("row_lb", C.c_void_p), ("row_ub", C.c_void_p), ("rii", C.c_void_p),
                ("col_type", C.c_void_p), ("col_lb", C.c_void_p), ("col_ub", C.c_void_p),
                ("col_coef", C.c_void_p), ("sjj", C.c_void_p),
                ("A_ptr", C.c_void_p), ("A_ind", C.c_void_p), ("A_val", C.c_void_p),
                ("a_version", C.c_ulonglong),
                ("head", C.c_void_p), ("row_stat", C.c_void_p), ("col_stat", C.c_void_p),
                ("row_bind", C.c_void_p), ("col_bind", C.c_void_p),
                ("row_prim", C.c_void_p), ("row_dual", C.c_void_p), ("col_prim", C.c_void_p),
                ("col_dual", C.c_void_p),
                ("it_cnt", C.c_int), ("pbs_stat", C.c_int), ("dbs_stat", C.c_int), ("some", C.c_int),
                ("obj_val", C.c_double), ("valid", C.c_int), ("b_version", C.c_ulonglong)]


class Iocp(C.Structure):
    _fields_ = [("msg_lev", C.c_int), ("br_tech", C.c_int), ("bt_tech", C.c_int), ("tol_int", C.c_double),
                ("tol_obj", C.c_double), ("tm_lim", C.c_int), ("out_frq", C.c_int), ("out_dly", C.c_int),
                ("pp_tech", C.c_int), ("mip_gap", C.c_double), ("presolve", C.c_int)]


class Mip(C.Structure):
    _fields_ = [("lp", Lp), ("col_kind", C.c_void_p), ("mip_stat", C.c_int), ("mip_obj", C.c_double),
                ("col_mipx", C.c_void_p), ("row_mipx", C.c_void_p), ("lp_solves", C.c_longlong),
                ("nodes_created", C.c_longlong), ("pivots", C.c_longlong), ("node_fallbacks", C.c_longlong),
                ("probe_lps", C.c_longlong), ("pp_fathomed", C.c_longlong), ("nodes_moved", C.c_longlong)]


_EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int)
_ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class IosShard(C.Structure):
    _fields_ = [("rank", C.c_int), ("size", C.c_int), ("ramp_nodes", C.c_int), ("sync_every", C.c_int),
                ("exchange", _EXCHANGE_FN), ("info", C.c_void_p), ("allgather", _ALLGATHER_FN)]


class SpxStats(C.Structure):
    _fields_ = [("pivots", C.c_longlong), ("reinversions", C.c_longlong), ("batches", C.c_longlong),
                ("host_syncs", C.c_longlong), ("seconds_total", C.c_double), ("seconds_reinvert", C.c_double),
                ("bytes_pivots", C.c_double), ("graphs_built", C.c_longlong),
                ("seconds_init", C.c_double), ("seconds_eval", C.c_double), ("seconds_batches", C.c_double),
                ("trow_ms", C.c_double), ("trow_launches", C.c_longlong), ("trow_bytes", C.c_double),
                ("trow_dev_ms", C.c_double), ("trow_dev_launches", C.c_longlong), ("trow_dev_ms_b", C.c_double),
                ("trow_dev_ms_r", C.c_double), ("trow_dev_launches_r", C.c_longlong),
                ("upd_dev_ms", C.c_double), ("upd_dev_launches", C.c_longlong), ("upd_bytes", C.c_double),
                ("resident", C.c_int), ("evals_skipped", C.c_int),
                ("panel_hits", C.c_longlong), ("panel_refills", C.c_longlong),
                ("refine_tries", C.c_longlong), ("refinements", C.c_longlong), ("refine_steps", C.c_longlong),
                ("refine_resid_max", C.c_double), ("factor_sparse", C.c_int), ("lu_ahead", C.c_int),
                ("seconds_lu", C.c_double), ("shard_exchanges", C.c_longlong)]


_lib = None

EXPORTS = ["gk_abi_version", "gk_device_count", "gk_ctx_create", "gk_ctx_destroy", "gk_last_error",
           "gk_bfd_create", "gk_bfd_destroy", "gk_bfd_set_parm", "gk_bfd_reset_parm", "gk_bfd_factorize", "gk_bfd_factorize_csc",
           "gk_bfd_ftran", "gk_bfd_btran", "gk_bfd_update", "gk_bfd_get_count", "gk_bfd_valid",
           "gk_spx_primal", "gk_spx_dual", "gk_bfd_last_stats", "gk_bfd_profile", "gk_ios_driver",
           "gk_scale_prob", "gk_scale_prob_timed", "gk_adv_basis", "gk_bfd_set_report",
           "gk_bfd_eval_tab_rows", "gk_ios_set_report", "gk_ios_driver_sharded", "gk_comm_create",
           "gk_comm_destroy", "gk_comm_backend", "gk_comm_rank", "gk_comm_size", "gk_comm_allgather",
           "gk_ios_driver_comm", "gk_comm_set_option", "gk_npp_create", "gk_npp_destroy", "gk_npp_load",
           "gk_npp_simplex", "gk_npp_integer", "gk_npp_build_size", "gk_npp_build", "gk_npp_postprocess",
           "gk_npp_unload_sol", "gk_npp_unload_mip", "gk_sp_selftest", "gk_comm_incumbent",
           "gk_comm_shared_incumbent", "gk_bfd_set_comm", "gk_build_stamp"]

# gk_report_fn (glpk_mi355x.h): one progress line or termination message of
# a gk_spx_* call, in the order the reference prints them
REPORT_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int)
_NULL_REPORT = REPORT_FN()


def load_library(path: str = LIB_PATH):
    """Load libglpk_mi355x.so; raises if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("GK_LIB_PATH", path)       # A/B experiments: another build of the library
    if not os.path.exists(path):
        raise GkError(f"{path} is missing: build it with __graft_entry__.build()")
    L = C.CDLL(path)
    P = C.c_void_p
    if hasattr(L, "gk_build_stamp"):
        L.gk_build_stamp.restype = C.c_char_p
    if "GK_LIB_PATH" not in os.environ and os.path.isdir(os.path.join(HERE, "csrc")):
        # the library must be the build of the sources beside it (stamp.py)
        from . import stamp as _stamp
        want, got = _stamp.source_stamp(), L.gk_build_stamp().decode()
        if got != want:
            raise GkError(f"{path} was built from other sources (stamp {got}, sources {want}): "
                          "rebuild it with __graft_entry__.build()")
    L.gk_abi_version.restype = C.c_int
    L.gk_device_count.restype = C.c_int
    L.gk_ctx_create.restype = P
    L.gk_ctx_create.argtypes = [C.c_int]
    L.gk_ctx_destroy.argtypes = [P]
    L.gk_last_error.restype = C.c_char_p
    L.gk_bfd_create.restype = P
    L.gk_bfd_create.argtypes = [P]
    L.gk_bfd_destroy.argtypes = [P]
    L.gk_bfd_set_parm.argtypes = [P, C.POINTER(Bfcp)]
    L.gk_bfd_set_parm.restype = C.c_int
    L.gk_bfd_reset_parm.argtypes = [P]
    L.gk_bfd_set_comm.argtypes = [P, P]
    L.gk_bfd_set_comm.restype = C.c_int
    L.gk_bfd_reset_parm.restype = C.c_int
    L.gk_bfd_factorize_csc.argtypes = [P, C.c_int, P, P, P]
    L.gk_bfd_factorize_csc.restype = C.c_int
    L.gk_bfd_ftran.argtypes = [P, P]
    L.gk_bfd_btran.argtypes = [P, P]
    L.gk_bfd_update.argtypes = [P, C.c_int, C.c_int, P, C.c_int, P]
    L.gk_bfd_update.restype = C.c_int
    L.gk_bfd_get_count.argtypes = [P]
    L.gk_bfd_get_count.restype = C.c_int
    L.gk_bfd_valid.argtypes = [P]
    L.gk_bfd_valid.restype = C.c_int
    for name in ("gk_spx_primal", "gk_spx_dual"):
        f = getattr(L, name)
        f.argtypes = [P, C.POINTER(Lp), P, C.POINTER(Smcp)]
        f.restype = C.c_int
    L.gk_bfd_last_stats.argtypes = [P, C.POINTER(SpxStats)]
    L.gk_ios_set_report.argtypes = [P, REPORT_FN, P]
    L.gk_comm_create.restype = P
    L.gk_comm_create.argtypes = [P, C.c_int, C.c_int, C.c_char_p, C.c_int]
    L.gk_comm_destroy.argtypes = [P]
    L.gk_comm_set_option.argtypes = [P, C.c_int, C.c_int]
    L.gk_comm_backend.argtypes = [P]
    L.gk_comm_allgather.argtypes = [P, P, C.c_size_t, P]
    L.gk_comm_allgather.restype = C.c_int
    L.gk_comm_incumbent.argtypes = [P, C.c_double]
    L.gk_comm_incumbent.restype = C.c_double
    L.gk_comm_shared_incumbent.argtypes = [P]
    L.gk_comm_shared_incumbent.restype = C.c_int
    L.gk_ios_driver_comm.argtypes = [P, C.POINTER(Mip), C.POINTER(Iocp), P]
    L.gk_ios_driver_comm.restype = C.c_int
    L.gk_ios_driver.argtypes = [P, C.POINTER(Mip), C.POINTER(Iocp)]
    L.gk_ios_driver.restype = C.c_int
    L.gk_ios_driver_sharded.argtypes = [P, C.POINTER(Mip), C.POINTER(Iocp), C.POINTER(IosShard)]
    L.gk_ios_driver_sharded.restype = C.c_int
    L.gk_bfd_profile.argtypes = [P, C.c_int]
    L.gk_bfd_profile.restype = None
    L.gk_ctx_mark.argtypes = [P, C.c_int]
    L.gk_ctx_mark.restype = C.c_int
    L.gk_bfd_trace.argtypes = [P, C.c_void_p, C.c_size_t]
    L.gk_bfd_trace.restype = C.c_int
    L.gk_bfd_time_kernel.argtypes = [P, C.c_int, C.c_int, C.POINTER(C.c_double)]
    L.gk_bfd_time_kernel.restype = C.c_double
    L.gk_scale_prob.argtypes = [P, C.c_int, C.c_int, P, P, P, C.c_int, P, P, P]
    L.gk_scale_prob.restype = C.c_int
    L.gk_scale_prob_timed.argtypes = [P, C.c_int, C.c_int, P, P, P, C.c_int, P, P, P, P, P]
    L.gk_scale_prob_timed.restype = C.c_int
    L.gk_adv_basis.argtypes = [P]
    L.gk_adv_basis.restype = C.c_int
    L.gk_bfd_set_report.argtypes = [P, REPORT_FN, P]
    L.gk_bfd_set_report.restype = None
    L.gk_bfd_eval_tab_rows.argtypes = [P, P, C.c_int, P, P, C.c_int]
    L.gk_bfd_eval_tab_rows.restype = C.c_int
    _lib = L
    return L


def _err(L) -> str:
    return L.gk_last_error().decode(errors="replace")


class Context:
    """One MI355X device (gk_ctx_create)."""

    def __init__(self, device: int = 0):
        self.L = load_library()
        self.h = self.L.gk_ctx_create(device)
        if not self.h:
            raise GkError(f"gk_ctx_create({device}) failed: {_err(self.L)}")

    def mark(self, tag: int):
        """Enqueue the marker kernel k_gk_mark (windows a kernel trace)."""
        self.L.gk_ctx_mark(self.h, int(tag))

    def close(self):
        if getattr(self, "h", None):
            self.L.gk_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


GK_COMM_AUTO, GK_COMM_TCP, GK_COMM_RCCL = 0, 1, 2


class Comm:
    """The library's collective for the sharded branch and bound
    (gk_comm_create): one per process, rank 0 listening on addr
    ("host:port"); RCCL when every rank has a device of its own (backend
    GK_COMM_AUTO), TCP through rank 0 otherwise.  ctx may be None for
    GK_COMM_TCP (no device)."""

    def __init__(self, ctx, rank: int, size: int, addr: str = "127.0.0.1:29533", backend: int = GK_COMM_AUTO):
        self.L = load_library()
        self.rank, self.size = int(rank), int(size)
        self.h = self.L.gk_comm_create(ctx.h if ctx is not None else None, self.rank, self.size,
                                       addr.encode(), int(backend))
        if not self.h:
            raise GkError(f"gk_comm_create failed: {_err(self.L)}")
        self.backend = self.L.gk_comm_backend(self.h)

    def allgather(self, block: bytes) -> list:
        """every rank's block (all the same size), rank order"""
        n = len(block)
        src = C.create_string_buffer(block, n)
        dst = C.create_string_buffer(n * self.size)
        if self.L.gk_comm_allgather(self.h, src, n, dst) != 0:
            raise GkError("gk_comm_allgather failed")
        raw = dst.raw
        return [raw[r * n:(r + 1) * n] for r in range(self.size)]

    @property
    def shared_incumbent(self) -> bool:
        """every rank on this host: the incumbent word in shared memory"""
        return bool(self.L.gk_comm_shared_incumbent(self.h))

    def incumbent(self, mine: float) -> float:
        """publish mine, return the best (minimum) published by any rank"""
        return float(self.L.gk_comm_incumbent(self.h, float(mine)))

    def close(self):
        if getattr(self, "h", None):
            self.L.gk_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def SMCP(**options) -> Smcp:
    """glpapi06.js:359-375, including the `options[x] || default` quirk:
    any falsy option (0) silently becomes the default."""
    d = dict(msg_lev=GLP_MSG_ALL, meth=GLP_PRIMAL, pricing=GLP_PT_PSE, r_test=GLP_RT_HAR, tol_bnd=1e-7,
             tol_dj=1e-7, tol_piv=1e-10, obj_ll=-DBL_MAX, obj_ul=+DBL_MAX, it_lim=INT_MAX, tm_lim=INT_MAX,
             out_frq=500, out_dly=0, presolve=0)
    for k, v in options.items():
        if k not in d:
            raise KeyError(k)
        if v:
            d[k] = v
    return Smcp(**d)


def _pad(a, dtype):
    out = np.zeros(len(a) + 1, dtype=dtype)
    out[1:] = a
    return out


class GkProblem:
    """The reference problem object's hot-path fields, 1-based, plus the
    device factor handle (lp.bfd) — what glp_simplex / glp_intopt operate on."""

    _version = 0

    def __init__(self, ctx: Context, p: Problem):
        self.ctx, self.L, self.p = ctx, ctx.L, p
        m, n = p.m, p.n
        self.m, self.n = m, n
        self.row_type = _pad(p.row_type, np.int8)
        self.row_lb = _pad(p.row_lb, np.float64)
        self.row_ub = _pad(p.row_ub, np.float64)
        self.rii = _pad(p.rii, np.float64)
        self.col_type = _pad(p.col_type, np.int8)
        self.col_lb = _pad(p.col_lb, np.float64)
        self.col_ub = _pad(p.col_ub, np.float64)
        self.col_coef = _pad(p.col_coef, np.float64)
        self.sjj = _pad(p.sjj, np.float64)
        self.col_kind = _pad(p.col_kind, np.int8)
        self.A_ptr = _pad(np.asarray(p.A_ptr, np.int32) + 1, np.int32)      # [1..n+1], 1-based positions
        self.A_ind = _pad(p.A_ind, np.int32)
        self.A_val = _pad(p.A_val, np.float64)
        self.row_stat = _pad(p.row_stat, np.int8)
        self.col_stat = _pad(p.col_stat, np.int8)
        self.head = np.zeros(m + 1, np.int32)
        self.row_bind = np.zeros(m + 1, np.int32)
        self.col_bind = np.zeros(n + 1, np.int32)
        self.row_prim = np.zeros(m + 1)
        self.row_dual = np.zeros(m + 1)
        self.col_prim = np.zeros(n + 1)
        self.col_dual = np.zeros(n + 1)
        self.dir, self.c0, self.nnz = p.dir, p.c0, p.nnz
        self.it_cnt = 0
        self.pbs_stat = self.dbs_stat = GLP_UNDEF
        self.obj_val = 0.0
        self.some = 0
        self.valid = 0
        self.mip_stat = GLP_UNDEF
        self.mip_obj = 0.0
        self.col_mipx = np.zeros(n + 1)
        self.row_mipx = np.zeros(m + 1)
        self.mip_stats = {}
        GkProblem._version += 1
        self.a_version = GkProblem._version
        # bounds / types / costs / scale version (gk_lp.b_version): 0 = unknown,
        # the engine rebuilds init_csa's arrays and compares them with the
        # resident copy on every call.  A caller that does not change them
        # between calls (numpy arrays can be changed in place, so the Python
        # host cannot know by itself) may declare it with touch_bounds() and
        # must call it again after every change, as the JS shim does on every
        # mutator
        self.b_version = 0
        self.bfcp = None
        self.bfd = self.L.gk_bfd_create(ctx.h)
        if not self.bfd:
            raise GkError(_err(self.L))

    def __del__(self):
        if getattr(self, "bfd", None):
            self.L.gk_bfd_destroy(self.bfd)
            self.bfd = None

    def set_bfcp(self, **kw):
        """glp_set_bfcp (glpapi12.js:133).  With no arguments (glp_set_bfcp(lp,
        NULL)): the defaults, re-inversion interval left to the engine; with
        any argument the values hold exactly (nfs_max = 100 included)."""
        if not kw:
            if self.L.gk_bfd_reset_parm(self.bfd) != 0:
                raise GkError(_err(self.L))
            self.bfcp = None
            return
        b = Bfcp(type=1, lu_size=0, piv_tol=0.10, piv_lim=4, suhl=1, eps_tol=1e-15, max_gro=1e10,
                 nfs_max=100, upd_tol=1e-6, nrs_max=100, rs_size=0)
        for k, v in kw.items():
            setattr(b, k, v)
        if self.L.gk_bfd_set_parm(self.bfd, C.byref(b)) != 0:
            raise GkError(_err(self.L))
        self.bfcp = b

    def set_comm(self, comm):
        """Column-sharded pricing of this LP's dual simplex over comm
        (gk_bfd_set_comm): every rank makes the same calls on the
        same problem; None turns it off."""
        self._comm = comm
        if self.L.gk_bfd_set_comm(self.bfd, comm.h if comm is not None else None) != 0:
            raise GkError(_err(self.L))

    def touch_matrix(self):
        """Invalidate the device copy of A (the shim's version counter)."""
        GkProblem._version += 1
        self.a_version = GkProblem._version
        if self.b_version:
            self.touch_bounds()

    def touch_bounds(self):
        """Declare the current bounds, types, costs, dir, c0 and scale
        factors as one version (gk_lp.b_version): later calls with the same
        version skip init_csa's rebuild.  Call again after every change."""
        GkProblem._version += 1
        self.b_version = GkProblem._version

    # ------------------------------------------------------------------
    _LP_ARRAYS = ("row_type", "row_lb", "row_ub", "rii", "col_type", "col_lb", "col_ub", "col_coef", "sjj",
                  "A_ptr", "A_ind", "A_val", "head", "row_stat", "col_stat", "row_bind", "col_bind",
                  "row_prim", "row_dual", "col_prim", "col_dual")

    _LP_GET = operator.itemgetter(*_LP_ARRAYS)

    def _lp_struct(self) -> Lp:
        # the struct and its array pointers are kept while every array
        # attribute is the same object (a numpy array's data never moves; an
        # attribute rebound to another array fails the identity test): a
        # fresh ctypes pointer per field and call cost ~0.1 ms per
        # glp_simplex call, ~2.5 % of a C3 it_lim=100 step
        cache = self.__dict__.setdefault("_ptr_cache", {})
        arrs = GkProblem._LP_GET(self.__dict__)
        lp = cache.get("lp")
        if lp is None or not all(map(operator.is_, arrs, cache["arrs"])):
            lp = Lp()
            for name, arr in zip(self._LP_ARRAYS, arrs):
                setattr(lp, name, arr.ctypes.data)
            cache["lp"], cache["arrs"] = lp, arrs
        lp.m, lp.n, lp.nnz, lp.dir, lp.c0 = self.m, self.n, self.nnz, self.dir, self.c0
        lp.a_version = self.a_version
        lp.b_version = self.b_version
        lp.it_cnt = self.it_cnt
        lp.pbs_stat = lp.dbs_stat = lp.some = lp.valid = 0     # (outputs: as a fresh struct)
        lp.obj_val = 0.0
        return lp

    def _take(self, lp: Lp):
        self.it_cnt, self.pbs_stat, self.dbs_stat = lp.it_cnt, lp.pbs_stat, lp.dbs_stat
        self.some, self.obj_val, self.valid = lp.some, lp.obj_val, lp.valid

    def factorize(self) -> int:
        """glp_factorize (glpapi12.js:5): basis header from statuses, then
        bfd_factorize with the columns of (I | -R A S) (b_col, :7)."""
        m, n = self.m, self.n
        self.valid = 0
        j = 0
        self.row_bind[:] = 0
        self.col_bind[:] = 0
        for k in range(1, m + n + 1):
            stat = self.row_stat[k] if k <= m else self.col_stat[k - m]
            if stat == GLP_BS:
                j += 1
                if j > m:
                    return GLP_EBADB
                self.head[j] = k
                if k <= m:
                    self.row_bind[k] = j
                else:
                    self.col_bind[k - m] = j
        if j < m:
            return GLP_EBADB
        if m > 0:
            ptr = np.zeros(m + 2, np.int32)
            ind, val = [0], [0.0]
            ptr[1] = 1
            for jj in range(1, m + 1):
                k = self.head[jj]
                if k <= m:
                    ind.append(k)
                    val.append(1.0)
                else:
                    c = k - m
                    lo, hi = self.A_ptr[c], self.A_ptr[c + 1]
                    rows = self.A_ind[lo:hi]
                    ind.extend(rows.tolist())
                    val.extend((-self.rii[rows] * self.A_val[lo:hi] * self.sjj[c]).tolist())
                ptr[jj + 1] = len(ind)
            ind = np.asarray(ind, np.int32)
            val = np.asarray(val, np.float64)
            ret = self.L.gk_bfd_factorize_csc(self.bfd, m, ptr.ctypes.data_as(C.c_void_p),
                                              ind.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p))
            if ret == GK_EABI:
                raise GkError(_err(self.L))
            if ret == 1:
                return GLP_ESING
            if ret == 2:
                return GLP_ECOND
            self.valid = 1
        return 0

    def ftran(self, x: np.ndarray, tr: bool = False) -> np.ndarray:
        """glp_ftran / glp_btran (glpapi12.js:198/:222) with the scaling."""
        m = self.m
        y = np.zeros(m + 1)
        y[1:] = x
        if not tr:
            y[1:] *= self.rii[1:]
            self.L.gk_bfd_ftran(self.bfd, y.ctypes.data_as(C.c_void_p))
            for i in range(1, m + 1):
                k = self.head[i]
                y[i] = y[i] / self.rii[k] if k <= m else y[i] * self.sjj[k - m]
        else:
            for i in range(1, m + 1):
                k = self.head[i]
                y[i] = y[i] / self.rii[k] if k <= m else y[i] * self.sjj[k - m]
            self.L.gk_bfd_btran(self.bfd, y.ctypes.data_as(C.c_void_p))
            y[1:] *= self.rii[1:]
        return y[1:]

    def spx(self, parm: Smcp, dual: bool) -> int:
        lp = self._lp_struct()
        fn = self.L.gk_spx_dual if dual else self.L.gk_spx_primal
        # one report callback per problem (a ctypes callback made per call
        # costs as much as a fresh pointer per field)
        if "_rpt_cb" not in self.__dict__:
            box = []                         # the callback holds the list, not self (no cycle)
            self._reports = box
            self._rpt_cb = REPORT_FN(lambda ud, *r: box.append(r))
        reports = self._reports
        reports.clear()
        self.L.gk_bfd_set_report(self.bfd, self._rpt_cb, None)
        try:
            ret = fn(self.ctx.h, C.byref(lp), self.bfd, C.byref(parm))
        finally:
            self.L.gk_bfd_set_report(self.bfd, _NULL_REPORT, None)
        # the display lines and messages (glpspx01.js:1587, glpspx02.js:1493),
        # printed in order after the solve
        for r in reports:
            for line in report_lines(*r):
                _xprintf(line)
        if ret == GK_EABI:
            raise GkError(_err(self.L))
        self._take(lp)
        return ret

    def eval_tab_rows(self, ks, per_row: bool = False) -> np.ndarray:
        """Rows of the simplex tableau of the basic variables ks (1..m+n) on
        the current factor, one GEMM for the batch (gk_bfd_eval_tab_rows;
        per_row: the CSC path): a (len(ks), m + n) array, column k - 1 =
        alfa of variable k (0 for basic variables), glp_eval_tab_row's
        values (glpapi12.js:401)."""
        ks = np.ascontiguousarray(ks, dtype=np.int32)
        out = np.zeros((len(ks), self.m + self.n))
        if len(ks) == 0:
            return out
        lp = self._lp_struct()
        ret = self.L.gk_bfd_eval_tab_rows(self.bfd, C.byref(lp), len(ks), ks.ctypes.data_as(C.c_void_p),
                                          out.ctypes.data_as(C.c_void_p), 1 if per_row else 0)
        if ret != 0:
            raise GkError(_err(self.L))
        return out

    def time_kernel(self, which: int, reps: int = 10):
        """(ms per launch, algorithmic bytes per launch) of one engine kernel,
        timed with HIP events on the engine stream (gk_bfd_time_kernel)."""
        b = C.c_double(0.0)
        ms = self.L.gk_bfd_time_kernel(self.bfd, which, reps, C.byref(b))
        if ms < 0:
            raise GkError(_err(self.L))
        return ms, b.value

    def profile(self, enable=True):
        """Record HIP events around the pivot-row kernel of every dual pivot
        (enable == 2: also per-block device clock stamps, see trace(); 3:
        the stamps only, inside the replayed graphs; 4: kernel spans and
        algorithmic bytes only, graphs kept — the bench's roofline pass)."""
        self.L.gk_bfd_profile(self.bfd, enable if enable in (2, 3, 4) else (1 if enable else 0))

    def trace(self) -> np.ndarray:
        """Per-kernel, per-block [entry, exit] device clock stamps of the last
        pivot (profile(2)); shape (8 kernels, 2048 blocks, 2).  The phase
        stamps that follow them are kept in self.trace_raw."""
        out = np.zeros(8 * 2048 * 10, dtype=np.uint64)
        self.L.gk_bfd_trace(self.bfd, out.ctypes.data_as(C.c_void_p), out.size)
        self.trace_raw = out
        return out[:8 * 2048 * 2].reshape(8, 2048, 2)

    def stats(self) -> SpxStats:
        st = SpxStats()
        self.L.gk_bfd_last_stats(self.bfd, C.byref(st))
        return st

    # ------------------------------------------------------------------
    def result(self) -> dict:
        return dict(pbs_stat=self.pbs_stat, dbs_stat=self.dbs_stat, obj_val=self.obj_val, it_cnt=self.it_cnt,
                    some=self.some, row_stat=self.row_stat[1:].copy(), col_stat=self.col_stat[1:].copy(),
                    row_prim=self.row_prim[1:].copy(), col_prim=self.col_prim[1:].copy(),
                    row_dual=self.row_dual[1:].copy(), col_dual=self.col_dual[1:].copy())


def _trivial_lp(P: GkProblem, parm: Smcp):
    """glpapi06.js:149."""
    P.valid = 0
    P.pbs_stat = P.dbs_stat = GLP_FEAS
    P.obj_val = P.c0
    P.some = 0
    p_infeas = d_infeas = 0.0
    for i in range(1, P.m + 1):
        t = P.row_type[i]
        P.row_stat[i] = GLP_BS
        P.row_prim[i] = P.row_dual[i] = 0.0
        if t in (GLP_LO, GLP_DB, GLP_FX) and P.row_lb[i] > +parm.tol_bnd:
            P.pbs_stat = GLP_NOFEAS
            if P.some == 0 and parm.meth != GLP_PRIMAL:
                P.some = i
        if t in (GLP_LO, GLP_DB, GLP_FX):
            p_infeas = max(p_infeas, P.row_lb[i])
        if t in (GLP_UP, GLP_DB, GLP_FX) and P.row_ub[i] < -parm.tol_bnd:
            P.pbs_stat = GLP_NOFEAS
            if P.some == 0 and parm.meth != GLP_PRIMAL:
                P.some = i
        if t in (GLP_UP, GLP_DB, GLP_FX):
            p_infeas = max(p_infeas, -P.row_ub[i])
    zeta = 1.0
    for j in range(1, P.n + 1):
        zeta = max(zeta, abs(P.col_coef[j]))
    zeta = (1.0 if P.dir == GLP_MIN else -1.0) / zeta
    for j in range(1, P.n + 1):
        t, coef = P.col_type[j], P.col_coef[j]
        if t == GLP_FR:
            P.col_stat[j], P.col_prim[j] = GLP_NF, 0.0
        elif t == GLP_LO:
            P.col_stat[j], P.col_prim[j] = GLP_NL, P.col_lb[j]
        elif t == GLP_UP:
            P.col_stat[j], P.col_prim[j] = GLP_NU, P.col_ub[j]
        elif t == GLP_DB:
            if zeta * coef > 0.0 or (zeta * coef == 0.0 and abs(P.col_lb[j]) <= abs(P.col_ub[j])):
                P.col_stat[j], P.col_prim[j] = GLP_NL, P.col_lb[j]
            else:
                P.col_stat[j], P.col_prim[j] = GLP_NU, P.col_ub[j]
        else:
            P.col_stat[j], P.col_prim[j] = GLP_NS, P.col_lb[j]
        P.col_dual[j] = coef
        P.obj_val += coef * P.col_prim[j]
        if t in (GLP_FR, GLP_LO) and zeta * coef < -parm.tol_dj:
            P.dbs_stat = GLP_NOFEAS
            if P.some == 0 and parm.meth == GLP_PRIMAL:
                P.some = P.m + j
        if t in (GLP_FR, GLP_LO):
            d_infeas = max(d_infeas, -zeta * coef)
        if t in (GLP_FR, GLP_UP) and zeta * coef > +parm.tol_dj:
            P.dbs_stat = GLP_NOFEAS
            if P.some == 0 and parm.meth == GLP_PRIMAL:
                P.some = P.m + j
        if t in (GLP_FR, GLP_UP):
            d_infeas = max(d_infeas, zeta * coef)
    # the simulated solver output (glpapi06.js:244-256)
    if parm.msg_lev >= GLP_MSG_ON and parm.out_dly == 0:
        inf = p_infeas if parm.meth == GLP_PRIMAL else d_infeas
        _xprintf(f"~{P.it_cnt}: obj = {_js_num(P.obj_val)}  infeas = {_js_num(inf)}")
    if parm.msg_lev >= GLP_MSG_ALL and parm.out_dly == 0:
        if P.pbs_stat == GLP_FEAS and P.dbs_stat == GLP_FEAS:
            _xprintf("OPTIMAL SOLUTION FOUND")
        elif P.pbs_stat == GLP_NOFEAS:
            _xprintf("PROBLEM HAS NO FEASIBLE SOLUTION")
        elif parm.meth == GLP_PRIMAL:
            _xprintf("PROBLEM HAS UNBOUNDED SOLUTION")
        else:
            _xprintf("PROBLEM HAS NO DUAL FEASIBLE SOLUTION")


def glp_eval_tab_row(P: GkProblem, k: int):
    """glp_eval_tab_row (glpapi12.js:401): the non-zeros of the tableau row of
    basic variable k as (ind, val) lists, variables in ascending order."""
    if not (P.m == 0 or P.valid):
        raise GkError("glp_eval_tab_row: basis factorization does not exist")
    if not (1 <= k <= P.m + P.n):
        raise GkError(f"glp_eval_tab_row: k = {k}; variable number out of range")
    row = P.eval_tab_rows([k])[0]
    ind = np.nonzero(row)[0]
    return (ind + 1).tolist(), row[ind].tolist()


def glp_simplex(P: GkProblem, parm: Smcp | None = None) -> int:
    """glp_simplex (glpapi06.js:1); presolve = GLP_ON runs the native
    preprocessor (presolve.preprocess_and_solve_lp, glpapi06.js:41)."""
    if parm is None:
        parm = SMCP()
    if parm.msg_lev not in (0, 1, 2, 3, 4):
        raise GkError(f"glp_simplex: msg_lev = {parm.msg_lev}; invalid parameter")
    if parm.meth not in (GLP_PRIMAL, GLP_DUALP, GLP_DUAL):
        raise GkError(f"glp_simplex: meth = {parm.meth}; invalid parameter")
    if parm.pricing not in (GLP_PT_STD, GLP_PT_PSE):
        raise GkError(f"glp_simplex: pricing = {parm.pricing}; invalid parameter")
    if parm.r_test not in (GLP_RT_STD, GLP_RT_HAR):
        raise GkError(f"glp_simplex: r_test = {parm.r_test}; invalid parameter")
    for name in ("tol_bnd", "tol_dj", "tol_piv"):
        v = getattr(parm, name)
        if not (0.0 < v < 1.0):
            raise GkError(f"glp_simplex: {name} = {v}; invalid parameter")
    if parm.it_lim < 0 or parm.tm_lim < 0 or parm.out_frq < 1 or parm.out_dly < 0:
        raise GkError("glp_simplex: invalid it_lim/tm_lim/out_frq/out_dly")
    if parm.presolve not in (0, 1):
        raise GkError(f"glp_simplex: presolve = {parm.presolve}; invalid parameter")
    P.pbs_stat = P.dbs_stat = GLP_UNDEF
    P.obj_val = 0.0
    P.some = 0
    # the double-bound check (glpapi06.js:306-323) runs once per bounds
    # version when the caller declares one (touch_bounds), on every call else
    bv = getattr(P, "b_version", 0)
    checked = bv != 0 and P.__dict__.get("_db_checked") == bv
    for what, typ, lb, ub in (() if checked else
                              (("row", P.row_type, P.row_lb, P.row_ub), ("column", P.col_type, P.col_lb, P.col_ub))):
        bad = np.nonzero((typ[1:] == GLP_DB) & (lb[1:] >= ub[1:]))[0]
        if bad.size:
            k = int(bad[0]) + 1
            if parm.msg_lev >= GLP_MSG_ERR:
                _xprintf(f"glp_simplex: {what} {k}: lb = {_js_num(lb[k])}, ub = {_js_num(ub[k])}; incorrect bounds")
            return GLP_EBOUND
    if bv:
        P._db_checked = bv
    if parm.msg_lev >= GLP_MSG_ALL:
        _xprintf(f"GLPK Simplex Optimizer, v{GLP_VERSION}")
        _xprintf(f"{P.m} row{'' if P.m == 1 else 's'}, {P.n} column{'' if P.n == 1 else 's'}, "
                 f"{P.nnz} non-zero{'' if P.nnz == 1 else 's'}")
    if P.nnz == 0:
        _trivial_lp(P, parm)
        return 0
    if parm.presolve:
        from . import presolve
        return presolve.preprocess_and_solve_lp(P, parm)
    return _solve_lp(P, parm)


def _solve_lp(P: GkProblem, parm: Smcp) -> int:
    """solve_lp (glpapi06.js:3): factorize if needed, then the method."""
    if not (P.m == 0 or P.valid):
        ret = P.factorize()
        if ret != 0:
            if parm.msg_lev >= GLP_MSG_ERR:
                _xprintf({GLP_EBADB: "glp_simplex: initial basis is invalid",
                          GLP_ESING: "glp_simplex: initial basis is singular",
                          GLP_ECOND: "glp_simplex: initial basis is ill-conditioned"}[ret])
            return ret
    if parm.meth == GLP_PRIMAL:
        return P.spx(parm, dual=False)
    if parm.meth == GLP_DUALP:
        ret = P.spx(parm, dual=True)
        if ret == GLP_EFAIL and P.valid:
            ret = P.spx(parm, dual=False)
        return ret
    return P.spx(parm, dual=True)


# ---------------------------------------------------------------------------
# glp_intopt (glpapi09.js:61-389) with presolve OFF and cb_func == null;
# ios_driver (glpios03.js:1) runs as gk_ios_driver on the MI355X
# ---------------------------------------------------------------------------
GLP_BR_FFV, GLP_BR_LFV, GLP_BR_MFV, GLP_BR_DTH, GLP_BR_PCH = 1, 2, 3, 4, 5
GLP_BT_DFS, GLP_BT_BFS, GLP_BT_BLB, GLP_BT_BPH = 1, 2, 3, 4
GLP_PP_NONE, GLP_PP_ROOT, GLP_PP_ALL = 0, 1, 2
GLP_EROOT, GLP_ENOPFS, GLP_ENODFS, GLP_EMIPGAP = 0x0C, 0x0A, 0x0B, 0x0E
GLP_CV, GLP_IV = 1, 2
GLP_OPT = 5


def IOCP(**options) -> Iocp:
    """IOCP (glpapi09.js:392-414), including its `options[x] || default` quirk."""
    d = dict(msg_lev=GLP_MSG_ALL, br_tech=GLP_BR_DTH, bt_tech=GLP_BT_BLB, tol_int=1e-5, tol_obj=1e-7,
             tm_lim=INT_MAX, out_frq=5000, out_dly=10000, pp_tech=GLP_PP_ALL, mip_gap=0.0, presolve=0)
    p = Iocp()
    for k, v in d.items():
        setattr(p, k, options.get(k) or v)
    # binarize (GLP_ON / GLP_OFF) steers only the host's presolve path
    p.binarize = options.get("binarize") or 0
    return p


def glp_intopt(P: GkProblem, parm: Iocp | None = None, comm=None, ramp_nodes: int = 0) -> int:
    """glp_intopt (glpapi09.js:61) -> solve_mip (:62) -> ios_driver.

    comm (shard.TorchComm or alike, size > 1): this process explores its share
    of the tree on its GPU; the incumbent and open nodes are exchanged through
    comm (an all-gather per sync epoch) and the best incumbent over all ranks
    is returned on every rank.  ramp_nodes: frontier per rank before the
    split (0: the driver's default; < 0: split the root alone, so that rank 0
    starts with all the work — a test of the open-node exchange)."""
    if parm is None:
        parm = IOCP()
    if parm.msg_lev not in (0, 1, 2, 3, 4):
        raise GkError(f"glp_intopt: msg_lev = {parm.msg_lev}; invalid parameter")
    if parm.br_tech not in (1, 2, 3, 4, 5):
        raise GkError(f"glp_intopt: br_tech = {parm.br_tech}; invalid parameter")
    if parm.bt_tech not in (1, 2, 3, 4):
        raise GkError(f"glp_intopt: bt_tech = {parm.bt_tech}; invalid parameter")
    if not (0.0 < parm.tol_int < 1.0):
        raise GkError(f"glp_intopt: tol_int = {parm.tol_int}; invalid parameter")
    if not (0.0 < parm.tol_obj < 1.0):
        raise GkError(f"glp_intopt: tol_obj = {parm.tol_obj}; invalid parameter")
    if parm.tm_lim < 0 or parm.out_frq < 0 or parm.out_dly < 0:
        raise GkError("glp_intopt: invalid tm_lim/out_frq/out_dly")
    if parm.pp_tech not in (0, 1, 2):
        raise GkError(f"glp_intopt: pp_tech = {parm.pp_tech}; invalid parameter")
    if parm.mip_gap < 0.0:
        raise GkError(f"glp_intopt: mip_gap = {parm.mip_gap}; invalid parameter")
    if parm.presolve not in (0, 1):
        raise GkError(f"glp_intopt: presolve = {parm.presolve}; invalid parameter")
    binarize = int(getattr(parm, "binarize", 0) or 0)
    if binarize not in (0, 1):
        raise GkError(f"glp_intopt: binarize = {binarize}; invalid parameter")
    P.mip_stat = GLP_UNDEF
    P.mip_obj = 0.0
    if np.any((P.row_type[1:] == GLP_DB) & (P.row_lb[1:] >= P.row_ub[1:])) or \
            np.any((P.col_type[1:] == GLP_DB) & (P.col_lb[1:] >= P.col_ub[1:])):
        return GLP_EBOUND
    iv = P.col_kind[1:] == GLP_IV
    t = P.col_type[1:]
    lb, ub = P.col_lb[1:], P.col_ub[1:]
    if np.any(iv & np.isin(t, (GLP_LO, GLP_DB, GLP_FX)) & (lb != np.floor(lb))) or \
            np.any(iv & np.isin(t, (GLP_UP, GLP_DB)) & (ub != np.floor(ub))):
        return GLP_EBOUND
    if parm.msg_lev >= GLP_MSG_ALL:
        # glp_intopt's header (glpapi09.js:368-383)
        ni = int(np.count_nonzero(P.col_kind[1:] == GLP_IV))
        nb = int(np.count_nonzero((P.col_kind[1:] == GLP_IV) & (P.col_type[1:] == GLP_DB) & (P.col_lb[1:] == 0.0) &
                                  (P.col_ub[1:] == 1.0)))
        s = ("none of" if nb == 0 else "" if (ni == 1 and nb == 1) else "one of" if nb == 1 else
             "all of" if nb == ni else f"{nb} of")
        _xprintf(f"GLPK Integer Optimizer, v{GLP_VERSION}")
        _xprintf(f"{P.m} row{'' if P.m == 1 else 's'}, {P.n} column{'' if P.n == 1 else 's'}, "
                 f"{P.nnz} non-zero{'' if P.nnz == 1 else 's'}")
        _xprintf(f"{ni} integer variable{'' if ni == 1 else 's'}, {s} which {'is' if nb == 1 else 'are'} binary")
    if parm.presolve:
        from . import presolve
        return presolve.preprocess_and_solve_mip(P, parm, bool(binarize))
    return _solve_mip(P, parm, comm, ramp_nodes)


def _solve_mip(P: GkProblem, parm: Iocp, comm, ramp_nodes: int) -> int:
    """solve_mip (glpapi09.js:62-111): the search, then its closing messages."""
    ret = _intopt(P, parm, comm, ramp_nodes)
    # solve_mip's closing messages (glpapi09.js:80-111)
    if ret == 0 and parm.msg_lev >= GLP_MSG_ALL:
        _xprintf("INTEGER OPTIMAL SOLUTION FOUND" if P.mip_stat == GLP_OPT else "PROBLEM HAS NO INTEGER FEASIBLE SOLUTION")
    elif ret == GLP_EMIPGAP and parm.msg_lev >= GLP_MSG_ALL:
        _xprintf("RELATIVE MIP GAP TOLERANCE REACHED; SEARCH TERMINATED")
    elif ret == GLP_ETMLIM and parm.msg_lev >= GLP_MSG_ALL:
        _xprintf("TIME LIMIT EXCEEDED; SEARCH TERMINATED")
    elif ret == GLP_EFAIL and parm.msg_lev >= GLP_MSG_ERR:
        _xprintf("glp_intopt: cannot solve current LP relaxation")
    return ret


def _intopt(P: GkProblem, parm: Iocp, comm, ramp_nodes: int) -> int:
    # solve_mip: an optimal basis to the LP relaxation must be provided
    if not (P.valid and P.pbs_stat == GLP_FEAS and P.dbs_stat == GLP_FEAS):
        if parm.msg_lev >= GLP_MSG_ERR:
            _xprintf("glp_intopt: optimal basis to initial LP relaxation not provided")
        return GLP_EROOT
    if parm.msg_lev >= GLP_MSG_ALL:
        _xprintf("Integer optimization begins...")
    # show_progress lines of the native driver (glpios03.js:2-48), printed
    # after the search in the order they were reported
    lines = []
    rcb = REPORT_FN(lambda ud, kind, code, it, a, obj, bnd, d:
                    lines.append(mip_progress_line(P.dir, code, it, a, obj, bnd, d)))
    P.L.gk_ios_set_report(P.ctx.h, rcb, None)
    try:
        return _intopt_run(P, parm, comm, ramp_nodes)
    finally:
        P.L.gk_ios_set_report(P.ctx.h, REPORT_FN(), None)
        for s in lines:
            _xprintf(s)


def _intopt_run(P: GkProblem, parm: Iocp, comm, ramp_nodes: int) -> int:
    mip = Mip()
    mip.lp = P._lp_struct()
    mip.lp.pbs_stat, mip.lp.dbs_stat, mip.lp.obj_val = P.pbs_stat, P.dbs_stat, P.obj_val
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)
    mip.col_kind = ptr(P.col_kind)
    mip.col_mipx = ptr(P.col_mipx)
    mip.row_mipx = ptr(P.row_mipx)
    if isinstance(comm, Comm) and (comm.size > 1 or comm.backend == GK_COMM_RCCL):
        # the library's own collective: the sharded search and the agreement
        # on the winning incumbent in C (gk_ios_driver_comm)
        P.L.gk_comm_set_option(comm.h, 1, int(ramp_nodes))
        ret = P.L.gk_ios_driver_comm(P.ctx.h, C.byref(mip), C.byref(parm), comm.h)
        if ret == GK_EABI:
            raise GkError(_err(P.L))
        P.mip_stat = mip.mip_stat
        P.mip_obj = mip.mip_obj
        P.mip_stats = _mip_stats(mip)
        return ret
    if comm is None or comm.size == 1:
        ret = P.L.gk_ios_driver(P.ctx.h, C.byref(mip), C.byref(parm))
        if ret == GK_EABI:
            raise GkError(_err(P.L))
        P.mip_stat = mip.mip_stat
        P.mip_obj = mip.mip_obj
        P.mip_stats = _mip_stats(mip)
        return ret
    errors = []

    def exchange(_info, best, active):
        try:
            b, act = comm.exchange(best[0], active)
            best[0] = b
            return act
        except Exception as e:          # a failing collective must not unwind through C
            errors.append(e)
            return 0

    def allgather(_info, send, nbytes, recv):
        try:
            comm.allgather_bytes(send, nbytes, recv)
            return 0
        except Exception as e:
            errors.append(e)
            return 1

    cb = _EXCHANGE_FN(exchange)
    ag = _ALLGATHER_FN(allgather) if hasattr(comm, "allgather_bytes") else _ALLGATHER_FN()
    sh = IosShard(rank=comm.rank, size=comm.size, ramp_nodes=int(ramp_nodes), sync_every=0, exchange=cb, info=None,
                  allgather=ag)
    ret = P.L.gk_ios_driver_sharded(P.ctx.h, C.byref(mip), C.byref(parm), C.byref(sh))
    if errors:
        raise errors[0]
    if ret == GK_EABI:
        raise GkError(_err(P.L))
    sign = 1.0 if P.dir == GLP_MIN else -1.0
    have = mip.mip_stat == GLP_OPT
    local = sign * (mip.mip_obj - P.c0) if have else float("inf")
    x = np.concatenate([P.row_mipx[1:], P.col_mipx[1:]])
    win, found, xw, _ = comm.finalize(local, have, x)
    if found:
        P.mip_stat = GLP_OPT
        P.mip_obj = P.c0 + sign * win
        P.row_mipx[1:] = xw[:P.m]
        P.col_mipx[1:] = xw[P.m:]
    else:
        P.mip_stat = GLP_NOFEAS
        P.mip_obj = 0.0
    P.mip_stats = dict(lp_solves=int(comm.total(mip.lp_solves)), nodes_created=int(comm.total(mip.nodes_created)),
                       pivots=int(comm.total(mip.pivots)), local_lp_solves=mip.lp_solves,
                       node_fallbacks=int(comm.total(mip.node_fallbacks)), probe_lps=int(comm.total(mip.probe_lps)),
                       pp_fathomed=int(comm.total(mip.pp_fathomed)), local_nodes_moved=mip.nodes_moved)
    return ret


def _mip_stats(mip) -> dict:
    return dict(lp_solves=mip.lp_solves, nodes_created=mip.nodes_created, pivots=mip.pivots,
                node_fallbacks=mip.node_fallbacks, probe_lps=mip.probe_lps, pp_fathomed=mip.pp_fathomed)


# ---------------------------------------------------------------------------
# glp_scale_prob (glpscl.js:1-225) — the factors come from the device
# (gk_scale_prob, gk_scale.hip); the host validates the flags, prints the
# reference's report lines and stores the factors like glp_set_rii /
# glp_set_sjj (glpapi04.js:1-28).
# ---------------------------------------------------------------------------
GLP_SF_GM, GLP_SF_EQ, GLP_SF_2N, GLP_SF_SKIP, GLP_SF_AUTO = 0x01, 0x10, 0x20, 0x40, 0x80

_print_func = None


def glp_set_print_func(f) -> None:
    """The reference's glp_set_print_func: every xprintf line goes to f (None:
    stdout)."""
    global _print_func
    _print_func = f


def _xprintf(s: str) -> None:
    if _print_func is not None:
        _print_func(s)
    else:
        print(s)


_REPORT_MSG = {1: "OPTIMAL SOLUTION FOUND", 2: "PROBLEM HAS NO DUAL FEASIBLE SOLUTION",
               3: "PROBLEM HAS NO FEASIBLE SOLUTION", 4: "PROBLEM HAS UNBOUNDED SOLUTION",
               5: "ITERATION LIMIT EXCEEDED; SEARCH TERMINATED", 6: "TIME LIMIT EXCEEDED; SEARCH TERMINATED",
               7: "OBJECTIVE LOWER LIMIT REACHED; SEARCH TERMINATED",
               8: "OBJECTIVE UPPER LIMIT REACHED; SEARCH TERMINATED",
               10: "Error: unable to choose basic variable on phase I"}


def report_lines(kind, code, it, phase, obj, inf, aux) -> list:
    """The lines the reference prints for one gk_report_fn record: the display
    lines of glpspx01.js:1587 (primal) and glpspx02.js:1493-1495 (dual), the
    termination messages of glpspx01.js:1815-1886 / glpspx02.js:1668-1886."""
    if kind == 1:
        if code == 1:
            return [f"{' ' if phase == 1 else '*'}{it}: obj = {_js_num(obj)}  infeas = {_js_num(inf)} ({aux})"]
        if phase == 1:
            return [f" {it}:  infeas = {_js_num(inf)} ({aux})"]
        return [f"|{it}: obj = {_js_num(obj)}  infeas = {_js_num(inf)} ({aux})"]
    if code == 9:
        return [f"Warning: numerical instability ({'primal' if aux == 1 else 'dual'} simplex, "
                f"phase {'I' if phase == 1 else 'II'})"]
    if code == 11:
        return [f"Error: unable to factorize the basis matrix ({aux})",
                "Sorry, basis recovery procedure not implemented yet"]
    return [_REPORT_MSG[code]] if code in _REPORT_MSG else []


def mip_progress_line(dir_, code, it, a_cnt, obj, bnd, deleted) -> str:
    """show_progress (glpios03.js:2-48) for one GK_RPT_MIP record."""
    from decimal import Decimal, ROUND_HALF_UP
    have, empty = bool(code & 2), bool(code & 4)
    best_mip = _js_num(obj) if have else "not found yet"
    if empty:
        best_bound = "tree is empty"
    elif bnd <= -1.7976931348623157e308:
        best_bound = "-inf"
    elif bnd >= 1.7976931348623157e308:
        best_bound = "+inf"
    else:
        best_bound = _js_num(bnd)
    rho = ">=" if dir_ == GLP_MIN else "<="
    # ios_relative_gap (glpios01.js:842)
    if not have:
        gap = 1.7976931348623157e308
    elif empty:
        gap = 0.0
    else:
        gap = abs(obj - bnd) / (abs(obj) + 2.220446049250313e-16)
    if gap == 0.0:
        rel = "  0.0%"
    elif gap < 0.001:
        rel = " < 0.1%"
    elif gap <= 9.999:
        # Number.prototype.toFixed(1): the nearest, the larger on a tie
        rel = "  " + str(Decimal(100.0 * gap).quantize(Decimal("0.1"), rounding=ROUND_HALF_UP)) + "%"
    else:
        rel = ""
    return (f"+{it}: {'>>>>>' if code & 1 else 'mip ='} {best_mip} {rho} {best_bound} {rel} "
            f"({a_cnt}; {deleted})")


def _js_num(x: float) -> str:
    """A double as JavaScript's Number.prototype.toString prints it (the
    shortest round-trip digits, JS's choice between plain and exponent form)."""
    x = float(x)
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))
    mant, _, exp = r.partition("e")
    e10 = int(exp) if exp else 0
    ip, _, fp = mant.partition(".")
    if fp == "0":
        fp = ""
    digits = (ip + fp).lstrip("0")
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    nexp = len(ip) + e10 - lead_zeros          # value = 0.digits * 10^nexp
    digits = digits.rstrip("0")
    k = len(digits)
    if k <= nexp <= 21:
        out = digits + "0" * (nexp - k)
    elif 0 < nexp <= 21:
        out = digits[:nexp] + "." + digits[nexp:]
    elif -6 < nexp <= 0:
        out = "0." + "0" * (-nexp) + digits
    else:
        e = nexp - 1
        out = digits[0] + ("." + digits[1:] if k > 1 else "") + "e" + ("+" if e > 0 else "-") + str(abs(e))
    return sign + out


class ScaleError(ValueError):
    """glp_scale_prob's xerror."""


def glp_scale_prob(P: GkProblem, flags: int) -> dict:
    """glp_scale_prob(lp, flags) (glpscl.js:215-225): the factors on the
    device, the report lines through the print function; returns the stage
    numbers {stage: (min, max, ratio)}."""
    flags = int(flags)
    if flags & ~(GLP_SF_GM | GLP_SF_EQ | GLP_SF_2N | GLP_SF_SKIP | GLP_SF_AUTO):
        raise ScaleError(f"glp_scale_prob: flags = {flags}; invalid scaling options")
    m, n = P.m, P.n
    ptr = np.ascontiguousarray(np.asarray(P.p.A_ptr, np.int32))
    ind = np.ascontiguousarray(np.asarray(P.p.A_ind, np.int32))
    val = np.ascontiguousarray(np.asarray(P.p.A_val, np.float64))
    rii, sjj, rep = np.ones(max(m, 1)), np.ones(max(n, 1)), np.zeros(13)
    f = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    ret = P.L.gk_scale_prob(P.ctx.h, m, n, f(ptr), f(ind), f(val), flags, f(rii), f(sjj), f(rep))
    if ret == 1:
        raise ScaleError(f"glp_scale_prob: flags = {flags}; invalid scaling options")
    if ret != 0:
        raise GkError(_err(P.L))
    bits = int(rep[12])
    _xprintf("Scaling...")
    stages = {}

    def line(tag, k):
        mn, mx, ratio = rep[3 * k: 3 * k + 3]
        stages[tag.strip()] = (mn, mx, ratio)
        _xprintf(f"{tag}: min|aij| = {_js_num(mn)}  max|aij| = {_js_num(mx)}  ratio = {_js_num(ratio)}")

    line(" A", 0)
    if bits & 1:
        _xprintf("Problem data seem to be well scaled")
    if not bits & 16:
        if bits & 2:
            line("GM", 1)
        if bits & 4:
            line("EQ", 2)
        if bits & 8:
            line("2N", 3)
    # glp_set_rii / glp_set_sjj: a change of a factor invalidates the basis
    # factorization when it touches a basic column (glpapi04.js:6-13, :23-26)
    old_r, old_s = P.rii[1:m + 1].copy(), P.sjj[1:n + 1].copy()
    new_r, new_s = rii[:m], sjj[:n]
    if P.valid:
        ch_r = (old_r != 1.0) | (new_r != 1.0)
        ch_s = (old_s != 1.0) | (new_s != 1.0)
        basic_c = np.asarray(P.col_stat[1:n + 1]) == GLP_BS
        if np.any(ch_s & basic_c):
            P.valid = 0
        elif np.any(ch_r):
            cols = np.repeat(np.arange(n), np.diff(ptr))
            rows = ind - 1
            if np.any(ch_r[rows] & basic_c[cols]):
                P.valid = 0
    P.rii[1:m + 1] = new_r
    P.sjj[1:n + 1] = new_s
    P.p.rii = new_r.copy()
    P.p.sjj = new_s.copy()
    P.touch_matrix()                              # the device copy of A is scaled: re-upload
    return stages


# ---------------------------------------------------------------------------
# glp_adv_basis (glpini01.js:1): the triangular starting basis (gk_adv_basis,
# host code in the library; no device needed)
# ---------------------------------------------------------------------------
def adv_basis_statuses(p, L=None):
    """gk_adv_basis on a problems.Problem: (size of the triangular part,
    row_stat[m], col_stat[n]) as the reference's adv_basis sets them."""
    L = L or load_library()
    m, n = p.m, p.n
    keep = dict(row_type=_pad(p.row_type, np.int8), row_lb=_pad(p.row_lb, np.float64),
                row_ub=_pad(p.row_ub, np.float64), col_type=_pad(p.col_type, np.int8),
                col_lb=_pad(p.col_lb, np.float64), col_ub=_pad(p.col_ub, np.float64),
                A_ptr=_pad(np.asarray(p.A_ptr, np.int32) + 1, np.int32), A_ind=_pad(p.A_ind, np.int32),
                row_stat=np.zeros(m + 1, np.int8), col_stat=np.zeros(n + 1, np.int8))
    f = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    lp = Lp()
    lp.m, lp.n, lp.nnz = m, n, p.nnz
    for k, v in keep.items():
        setattr(lp, k, f(v))
    ret = L.gk_adv_basis(C.byref(lp))
    if ret < 0:
        raise GkError(_err(L))
    return ret, keep["row_stat"][1:].copy(), keep["col_stat"][1:].copy()


def glp_adv_basis(P: "GkProblem", flags: int = 0, msg_lev: int = 3) -> int:
    """glp_adv_basis(lp, flags) (glpini01.js:356-362) on the Python host:
    the statuses of the triangular basis into P (the basis factorization is
    then invalid, as glp_set_row_stat / glp_set_col_stat leave it)."""
    if flags != 0:
        raise GkError(f"glp_adv_basis: flags = {flags}; invalid flags")
    if P.m == 0 or P.n == 0:
        size, rs, cs = adv_basis_statuses(P.p, P.L)
    else:
        _xprintf("Constructing initial basis...")
        size, rs, cs = adv_basis_statuses(P.p, P.L)
        if msg_lev >= 3:
            _xprintf(f"Size of triangular part = {size}")
    P.row_stat[1:P.m + 1] = rs
    P.col_stat[1:P.n + 1] = cs
    P.valid = 0
    return size
