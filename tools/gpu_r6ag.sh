# round 6 diagnostics: which GPU tests depend on memory never written
# (new device buffers poisoned with 0xff)
O=gpurun_out/${1:-r6ag}; mkdir -p $O
GK_DEBUG_POISON=0xff timeout -k 10 600 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_lp.py tests/test_gpu_mip.py tests/test_gpu_sparse.py -m gpu -x -k "not sharded" > $O/poison_ff.log 2>&1
echo "rc $?" >> $O/poison_ff.log
GK_DEBUG_POISON=0xff timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_lp.py -m gpu > $O/poison_ff_lp_all.log 2>&1
echo "rc $?" >> $O/poison_ff_lp_all.log
