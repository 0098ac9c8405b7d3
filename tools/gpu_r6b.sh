# round 6: the sharded dual's RCCL branch, the 12x42 fixture through the
# single-GPU and two-rank searches
O=gpurun_out/${1:-r6b}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lp_shard.py \
  "tests/test_gpu_mip.py::test_gpu_mip_matches_reference" tests/test_shard.py::test_sharded_bnb_two_ranks_one_gpu \
  "tests/test_comm.py" -s > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "
import sys, json; sys.path.insert(0, '.')
import torch, bench, __graft_entry__
__graft_entry__.load_package()
from glpk_js_amd import gk, problems
ctx = gk.Context(0)
print(json.dumps(bench.run_sparse(gk, problems, ctx)))
" > $O/sparse20k.json 2> $O/sparse20k.err || exit 2
