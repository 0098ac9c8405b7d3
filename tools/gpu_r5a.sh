# round-5 measurement set: sparse blocks-40 (default factor choice) and
# blocks-200 (m = 20,020) full solves, then the bench
O=gpurun_out/${1:-r5a}
mkdir -p $O
timeout -k 10 120 python3 -u tools/sparse_big.py blocks 40 5 > $O/blocks40_default.json 2> $O/blocks40.err || exit 1
timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/blocks200.json 2> $O/blocks200.err || exit 2
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 3
