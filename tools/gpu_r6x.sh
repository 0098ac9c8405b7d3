# round 6: pipelined inv(M) loads (k_sp_update, ftran_hh) — tests, profile, full solve
set -e
O=gpurun_out/${1:-r6x}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py tests/test_sparse_factor.py -m gpu > $O/tests.log 2>&1
bash tools/prof_sparse_window.sh r6x_spw20 --it 1000 --basis profiles/r06_blocks20k_basis_it61912.npz 200 20 > $O/spw.log 2>&1
timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/full20k.json 2> $O/full20k.err
timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 > $O/w100.json 2>/dev/null
echo ok
