# round 6: engine mode back to one node LP at a time by default — MIP tests
# twice (pinned counts), the sharded engine-mode tests, timings
set -e
O=gpurun_out/${1:-r6ae}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_mip.py tests/test_comm.py -m gpu > $O/mip1.log 2>&1 || { tail -30 $O/mip1.log; exit 1; }
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_mip.py -m gpu > $O/mip2.log 2>&1 || { tail -30 $O/mip2.log; exit 1; }
timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 sparsebig4 > $O/bnb.json 2> $O/bnb.err
echo ok
