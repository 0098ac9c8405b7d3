# small-factor sweeps with LDS-resident outputs (GK_SP_LDS): blocks-40 rate on / off, then the sparse tests
O=gpurun_out/${1:-splds}
mkdir -p $O
for v in 1 0; do
  GK_SP_LDS=$v timeout -k 10 200 python3 -u tools/sparse_big.py blocks 40 5 > $O/b40_$v.json 2> $O/b40_$v.err || exit 2
  echo "lds $v: $(tail -c 230 $O/b40_$v.json)"
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 4; }
tail -1 $O/t.txt
