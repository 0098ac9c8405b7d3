# round 6: k_dual_top block-split chuzr scan — sparse window m = 100k under
# rocprof, sparse tests; the m = 100k level histograms and launch plans
set -e
O=gpurun_out/${1:-r6r}; mkdir -p $O
bash tools/prof_sparse_window.sh r6r_spw --it 1000 > $O/spw.log 2>&1
GK_SP_LEVELS=1 timeout -k 10 200 python3 -u tools/sparse_window.py --it 5 > $O/levels100k.json 2> $O/levels100k.txt
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py tests/test_sparse_factor.py -m gpu > $O/tests.log 2>&1
echo ok
