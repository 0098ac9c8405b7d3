# sparse path: tests, pivot window (look-ahead on / off), per-level stamps
O=gpurun_out/${1:-s2}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --durations=8 --timeout 250 --timeout-method thread tests/test_gpu_sparse.py > $O/sparse_tests.txt 2>&1 || exit 2
GK_SPARSE_LOG=1 timeout -k 10 200 python3 -u tools/sparse_window.py --it 1000 > $O/win.json 2> $O/win.err || exit 3
GK_SP_AHEAD=0 timeout -k 10 200 python3 -u tools/sparse_window.py --it 1000 > $O/win_noahead.json 2>&1 || exit 4
GK_SP_STAMPS=$O/stamps.txt timeout -k 10 200 python3 -u tools/sparse_window.py --it 200 > $O/stamps_run.json 2>&1 || exit 5
