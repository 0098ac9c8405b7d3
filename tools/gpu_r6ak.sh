# round 6: the sparse windows' kernel statistics on the final tree
set -e
bash tools/prof_sparse_window.sh r6ak_100k --it 1000 > /dev/null 2>&1
bash tools/prof_sparse_window.sh r6ak_20k --it 1000 --basis profiles/r06_blocks20k_basis_it61912.npz 200 20 > /dev/null 2>&1
echo ok
