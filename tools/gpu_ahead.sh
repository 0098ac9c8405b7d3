# sparse m = 100k window: the look-ahead's lead (GK_SP_AHEAD) swept
O=gpurun_out/${1:-ahead}
mkdir -p $O
for a in 32 64 96; do
  GK_SPARSE_LOG=1 GK_SP_AHEAD=$a timeout -k 10 200 python3 -u tools/sparse_window.py --it 1000 > $O/win_$a.json 2> $O/win_$a.err || exit 3
  echo "ahead $a: $(tail -c 300 $O/win_$a.json)"
done
