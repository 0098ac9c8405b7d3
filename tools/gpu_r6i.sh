# round 6: sparse window without the pivot-row pass's max atomic, sparse + LP tests
O=gpurun_out/${1:-r6i}; mkdir -p $O
bash tools/prof_sparse_window.sh r6i_spw --it 1000 > $O/spw.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py tests/test_sparse_factor.py tests/test_gpu_lp.py tests/test_lp_shard.py tests/test_gpu_determinism.py -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
