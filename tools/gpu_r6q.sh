# round 6: re-pin the B&B counts and check them in the MIP tests
set -e
O=gpurun_out/${1:-r6q}; mkdir -p $O
timeout -k 10 400 python3 -u tools/bnb_counts.py gpurun_out/bnb_counts.json > $O/counts.log 2>&1
cp gpurun_out/bnb_counts.json tests/golden/bnb_counts.json
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_mip.py tests/test_shard.py tests/test_comm.py -m gpu > $O/mip.log 2>&1
echo ok
