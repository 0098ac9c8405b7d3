O=gpurun_out/${1:-r5c}
mkdir -p $O
timeout -k 10 120 python3 -u tools/sparse_big.py blocks 40 5 > $O/blocks40_default.json 2> $O/blocks40.err || exit 1
GK_SP_SEG=0 timeout -k 10 120 python3 -u tools/sparse_big.py blocks 40 5 > $O/blocks40_noseg.json 2>> $O/blocks40.err || exit 1
timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/blocks200.json 2> $O/blocks200.err || exit 3
GK_SP_SEG=0 timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/blocks200_noseg.json 2>> $O/blocks200.err || exit 3
