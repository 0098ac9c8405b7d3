# sparse factor at small m: blocks-40 and the m = 20,020 solve (rates), then the sparse tests
O=gpurun_out/${1:-spsmall}
mkdir -p $O
timeout -k 10 200 python3 -u tools/sparse_big.py blocks 40 5 > $O/b40.json 2> $O/b40.err || exit 2
echo "b40: $(tail -c 260 $O/b40.json)"
timeout -k 10 200 python3 -u tools/sparse_big.py blocks 200 20 > $O/b200.json 2> $O/b200.err || exit 3
echo "b200: $(tail -c 260 $O/b200.json)"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py > $O/t.txt 2>&1 || exit 4
tail -1 $O/t.txt
