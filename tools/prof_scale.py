#!/usr/bin/env python3
"""glp_scale_prob(GM | EQ | 2N) on C3 once (for rocprofv3 --kernel-trace):
usage: python tools/prof_scale.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402  (one HIP runtime: torch first)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402
import bench  # noqa: E402

ctx = gk.Context(0)
p = problems.gen_dense(4096, 16384, seed=42)
for _ in range(2):
    print(json.dumps(bench.run_scale(gk, ctx, p)))
