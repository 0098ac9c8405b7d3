# round 6: MIP / comm tests and smoke() on the final tree
O=gpurun_out/${1:-r6aj}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_mip.py tests/test_comm.py tests/test_shard.py -m gpu > $O/mip.log 2>&1
echo "rc $?" >> $O/mip.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc $?" >> $O/smoke.log
