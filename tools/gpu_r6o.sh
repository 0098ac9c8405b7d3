# round 6: pin the B&B counts (tools/bnb_counts.py) and check them with the
# MIP tests in a second process; the column-pass A/B (gpu_r6n.sh) before
set -e
O=gpurun_out/${1:-r6o}; mkdir -p $O
bash tools/gpu_r6n.sh > $O/r6n.log 2>&1
timeout -k 10 400 python3 -u tools/bnb_counts.py gpurun_out/bnb_counts.json > $O/counts.log 2>&1
cp gpurun_out/bnb_counts.json tests/golden/bnb_counts.json
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_mip.py -m gpu > $O/mip.log 2>&1
echo ok
