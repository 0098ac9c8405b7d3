# round 6: the sharded dual's RCCL branch, the 12x42 fixture through the
# single-GPU and two-rank searches
O=gpurun_out/${1:-r6b}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lp_shard.py \
  "tests/test_gpu_mip.py::test_gpu_mip_matches_reference" tests/test_shard.py::test_sharded_bnb_two_ranks_one_gpu \
  "tests/test_comm.py" -s > $O/tests.log 2>&1 || exit 1
