# sparse m = 20,020 full dual solve: default vs the look-ahead at this m (GK_SP_AHEAD_MIN_M) and its lead
O=gpurun_out/${1:-s20k}
mkdir -p $O
timeout -k 10 200 python3 -u tools/sparse_big.py blocks 200 20 > $O/base.json 2> $O/base.err || exit 2
echo "base: $(tail -c 260 $O/base.json)"
for a in 16 32; do
  GK_SP_AHEAD_MIN_M=10000 GK_SP_AHEAD=$a timeout -k 10 200 python3 -u tools/sparse_big.py blocks 200 20 > $O/ah$a.json 2> $O/ah$a.err || exit 3
  echo "ahead $a: $(tail -c 260 $O/ah$a.json)"
done
