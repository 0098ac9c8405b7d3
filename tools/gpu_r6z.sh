# round 6: inv(M)'s rank-1 update on k_sp_ycol's grid — tests, A/B against
# the HEAD library (glpk.js_amd/ab_head.so), full m = 20k solve
set -e
O=gpurun_out/${1:-r6z}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py tests/test_sparse_factor.py -m gpu > $O/tests.log 2>&1
B=profiles/r06_blocks20k_basis_it61912.npz
bash tools/prof_sparse_window.sh r6z_new --it 1000 --basis $B 200 20 > $O/pn.log 2>&1
GK_LIB_PATH=$GRAFT_REPO_ROOT/glpk.js_amd/ab_head.so bash tools/prof_sparse_window.sh r6z_old --it 1000 --basis $B 200 20 > $O/po.log 2>&1
timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/full20k.json 2> $O/full20k.err
echo ok
# (the m = 100k window both ways)
timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 > $O/w100_new.json 2>/dev/null
GK_LIB_PATH=$GRAFT_REPO_ROOT/glpk.js_amd/ab_head.so timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 > $O/w100_old.json 2>/dev/null
