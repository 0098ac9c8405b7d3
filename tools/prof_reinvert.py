#!/usr/bin/env python3
"""Re-inversion at a given k (gk_bfd_factorize_csc on an m x m basis with k
dense structural columns, as tests/test_gpu_factor.py builds them), checked
against numpy on one FTRAN.  Run under rocprofv3 --kernel-trace --stats for
the device time of the Gauss-Jordan kernels:

  rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/prof_reinvert.py 4096 4096"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk  # noqa: E402
from test_gpu_factor import _basis, _factorize  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    k = int(sys.argv[2]) if len(sys.argv) > 2 else m
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    ctx = gk.Context(0)
    L = gk.load_library()
    f = L.gk_bfd_create(ctx.h)
    B = _basis(m, k, 7)
    for r in range(reps):
        t0 = time.perf_counter()
        assert _factorize(f, L, B) == 0
        print(f"factorize {r}: {time.perf_counter() - t0:.3f} s (host wall, incl. CSC upload)")
    rng = np.random.default_rng(1)
    x = rng.standard_normal(m)
    y = np.zeros(m + 1)
    y[1:] = x
    L.gk_bfd_ftran(f, y.ctypes.data_as(C.c_void_p))
    ref = np.linalg.solve(B, x)
    err = np.max(np.abs(y[1:] - ref)) / max(1.0, np.max(np.abs(ref)))
    print(f"ftran max rel err vs numpy: {err:.2e}")
    assert err < 1e-8
    L.gk_bfd_destroy(f)


if __name__ == "__main__":
    main()
