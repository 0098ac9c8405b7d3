"""glpk.js_amd — MI355X-native revised-simplex and branch-and-bound core for
the Cyame/glpk.js (GLPK 4.49 JS) hot path.

The directory name contains a dot, so it is loaded as the module
``glpk_js_amd`` through ``load_package()`` in __graft_entry__.py.

Layout:
  csrc/        HIP kernels (gfx950) + C++ host driver + the C-ABI
               (include/glpk_mi355x.h), built into libglpk_mi355x.so
  problems.py  problem instances and the SURVEY.md §8(d) generators
  gk.py        ctypes binding of the C-ABI and the host-side mirror of
               glp_simplex / glp_intopt for Python callers and tests
"""
