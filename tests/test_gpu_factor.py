"""Re-inversion (gk_bfd_factorize_csc, the bfd_factorize of glpbfd.js:74) at
the sizes where the blocked Gauss-Jordan changes configuration (panel width
and rows per thread, gk_reinvert.hip), checked against numpy's solve: FTRAN
and BTRAN of random right-hand sides, and BFD_ESING on a singular basis."""
import ctypes as C

import numpy as np
import pytest

from glpk_js_amd import gk

pytestmark = pytest.mark.gpu


def _basis(m, k, seed):
    """m x m basis: k dense random columns over k random rows (plus a few
    entries in the slack rows), the other m - k columns unit (slacks)."""
    rng = np.random.default_rng(seed)
    B = np.zeros((m, m))
    slack_rows = rng.permutation(m)[: m - k]
    R = np.setdiff1d(np.arange(m), slack_rows)
    perm = rng.permutation(m)
    other_pos, struct_pos = perm[: m - k], perm[m - k:]
    for j, pos in enumerate(other_pos):
        B[slack_rows[j], pos] = 1.0
    for pos in struct_pos:
        B[R, pos] = rng.standard_normal(k)
        if m > k:
            extra = rng.choice(slack_rows, size=min(3, m - k), replace=False)
            B[extra, pos] = rng.standard_normal(len(extra))
    return B


def _factorize(P_bfd, L, B):
    m = B.shape[0]
    ptr = np.zeros(m + 2, np.int32)
    ind, val = [0], [0.0]
    ptr[1] = 1
    for j in range(m):
        nz = np.nonzero(B[:, j])[0]
        ind.extend((nz + 1).tolist())
        val.extend(B[nz, j].tolist())
        ptr[j + 2] = len(ind)
    ind = np.asarray(ind, np.int32)
    val = np.asarray(val, np.float64)
    return L.gk_bfd_factorize_csc(P_bfd, m, ptr.ctypes.data_as(C.c_void_p), ind.ctypes.data_as(C.c_void_p),
                                  val.ctypes.data_as(C.c_void_p))


@pytest.fixture(scope="module")
def bfd(gpu_ctx):
    L = gk.load_library()
    f = L.gk_bfd_create(gpu_ctx.h)
    assert f
    yield L, f
    L.gk_bfd_destroy(f)


@pytest.mark.parametrize("m,k", [(8, 1), (20, 20), (40, 16), (40, 17), (300, 256), (300, 257), (600, 512),
                                 (600, 513), (1100, 1024), (1100, 1025), (2100, 2049), (4096, 4096), (4200, 4097)])
def test_gpu_reinversion_sizes(bfd, m, k):
    L, f = bfd
    B = _basis(m, k, seed=m + k)
    assert _factorize(f, L, B) == 0
    rng = np.random.default_rng(k)
    for tr in (False, True):
        b = rng.standard_normal(m)
        y = np.zeros(m + 1)
        y[1:] = b
        (L.gk_bfd_btran if tr else L.gk_bfd_ftran)(f, y.ctypes.data_as(C.c_void_p))
        x = np.linalg.solve(B.T if tr else B, b)
        err = np.max(np.abs(y[1:] - x)) / (1.0 + np.max(np.abs(x)))
        assert err <= 1e-8, (m, k, tr, err)


def test_gpu_reinversion_singular(bfd):
    """Two equal structural columns (small basis), and a row of the
    structural block that is zero in every structural column (large basis:
    the pivot candidates of its step are exactly zero), give BFD_ESING."""
    L, f = bfd
    B = _basis(30, 20, seed=7)
    nz = np.nonzero(np.abs(B).sum(axis=0) > 1.0)[0]
    B[:, nz[-1]] = B[:, nz[0]]
    assert _factorize(f, L, B) == 1
    B = _basis(700, 600, seed=7)
    struct = np.nonzero(np.count_nonzero(B, axis=0) > 1)[0]
    row = int(np.nonzero(np.count_nonzero(B[:, struct], axis=1) == len(struct))[0][0])   # a row of C
    B[row, struct] = 0.0
    assert _factorize(f, L, B) == 1
