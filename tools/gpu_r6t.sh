# round 6: level stamps of the m = 20,020 mid-solve factor's sweeps
set -e
O=gpurun_out/${1:-r6t}; mkdir -p $O
GK_SP_STAMPS=$O/stamps20k.txt timeout -k 10 200 python3 -u tools/sparse_window.py --it 200 --basis profiles/r06_blocks20k_basis_it61912.npz 200 20 > $O/run.json 2>&1
echo ok
