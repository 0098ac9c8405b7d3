# round 6: concurrent engine-mode node LPs — MIP tests (pinned counts), timings
set -e
O=gpurun_out/${1:-r6ab}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_mip.py -m gpu > $O/mip.log 2>&1 || { tail -30 $O/mip.log; exit 1; }
timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 sparsebig2 sparsebig3 sparsebig4 > $O/bnb.json 2> $O/bnb.err
echo ok
