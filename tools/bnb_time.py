#!/usr/bin/env python3
"""glp_intopt on MIP fixtures (tests/golden/mip_<name>.json) as bench.py's
B&B legs time it: python tools/bnb_time.py [NAME ...] (default gap c5s_12x30)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
import __graft_entry__  # noqa: E402
import bench  # noqa: E402

__graft_entry__.load_package()
from glpk_js_amd import gk, problems  # noqa: E402

if __name__ == "__main__":
    names = tuple(sys.argv[1:]) or ("gap", "c5s_12x30")
    ctx = gk.Context(0)
    for name in names:
        print(json.dumps(bench.run_bnb(gk, problems, ctx, names=(name,))), flush=True)
