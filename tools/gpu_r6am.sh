# round 6: LP / determinism GPU tests and smoke() after the last engine change
O=gpurun_out/${1:-r6am}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_lp.py tests/test_gpu_determinism.py tests/test_lp_shard.py tests/test_gpu_mip.py -m gpu > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc $?" >> $O/smoke.log
