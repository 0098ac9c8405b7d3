# C3 mid-solve window with the pricing panel's size swept (GK_PANEL)
O=gpurun_out/${1:-psweep}
mkdir -p $O
for k in 32 16 0; do
  GK_PANEL=$k timeout -k 10 200 python3 -u tools/c3_mid.py 100000 30 > $O/mid_$k.txt 2>&1 || exit 2
  echo "panel $k: $(tail -1 $O/mid_$k.txt | cut -c1-260)"
done
