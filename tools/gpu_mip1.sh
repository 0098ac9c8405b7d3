O=gpurun_out/${1:-mip1}
mkdir -p $O
timeout -k 10 120 python3 -u tools/bnb_time.py c5s_12x40 c5s_12x38 > $O/deep.txt 2>&1 || exit 1
GK_BNB_CAP=1 GK_BNB_PRECAP=1 GK_BNB_DEPTH=1 timeout -k 10 120 python3 -u tools/bnb_time.py gap > $O/gap_seq.txt 2>&1 || exit 2
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_mip.py -k "12x38 or 12x40" > $O/mip_deep_tests.txt 2>&1 || exit 3
