# round 6: the sharded search in engine mode (2 TCP ranks on one GPU)
O=gpurun_out/${1:-r6ac}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_comm.py -k engine_mode -m gpu > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
