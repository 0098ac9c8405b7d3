# round 6: the m = 100k window by GK_SP_WIDE / GK_SP_GA (two runs each)
O=gpurun_out/${1:-r6aa}; mkdir -p $O
for rep in 1 2; do
  for wd in 4096 6144 8192; do
    for ga in 2048 1024; do
      GK_SP_GA=$ga GK_SP_WIDE=$wd timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 > $O/w100_wd${wd}_ga${ga}_$rep.json 2>/dev/null || exit 1
    done
  done
done
echo ok
