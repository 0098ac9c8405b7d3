O=gpurun_out/${1:-r5b}
mkdir -p $O
timeout -k 10 120 python3 -u tools/sparse_big.py blocks 40 5 > $O/blocks40_default.json 2> $O/blocks40.err || exit 1
for a in 32 48 64; do GK_SP_AHEAD=$a timeout -k 10 200 python3 -u tools/sparse_window.py --it 1000 > $O/win_ahead$a.json 2>&1 || exit 2; done
timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/blocks200.json 2> $O/blocks200.err || exit 3
