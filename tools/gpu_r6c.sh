# round 6: the two-kernel dual pivot (DualPlan.fold) — LP parity and
# determinism, the B&B engine mode, then the headline window with fold on and off
O=gpurun_out/${1:-r6c}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_lp.py \
  tests/test_gpu_determinism.py "tests/test_gpu_mip.py::test_gpu_mip_engine_mode" -s > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
timeout -k 10 200 python3 -u bench.py --no-cpu --no-extra > $O/bench_fold.json 2> $O/bench_fold.err || exit 2
GK_FOLD=0 timeout -k 10 200 python3 -u bench.py --no-cpu --no-extra > $O/bench_nofold.json 2> $O/bench_nofold.err || exit 3
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lp_shard.py -s > $O/shard.log 2>&1 || exit 4
