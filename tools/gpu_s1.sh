mkdir -p gpurun_out/s1
timeout -k 10 150 python3 -u tools/bnb_time.py gap c5s_12x30 c5s_12x32 c5s_12x34 > gpurun_out/s1/bnb.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_sparse.py > gpurun_out/s1/sparse_tests.txt 2>&1 || exit 2
timeout -k 10 200 python3 -u tools/sparse_window.py --it 1000 > gpurun_out/s1/win_seg.json 2>&1 || exit 3
GK_SP_SEG=0 timeout -k 10 200 python3 -u tools/sparse_window.py --it 1000 > gpurun_out/s1/win_noseg.json 2>&1 || exit 4
GK_SP_STAMPS=gpurun_out/s1/stamps.txt timeout -k 10 200 python3 -u tools/sparse_window.py --it 200 > gpurun_out/s1/stamps_run.json 2>&1 || exit 5
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_mip.py > gpurun_out/s1/mip_tests.txt 2>&1 || exit 6
