# round 6: sparse plan knobs (GK_SP_GA: external entries from which a
# segment's external pass runs on the grid; GK_SP_WIDE: steps from which a
# level runs on the grid) on the m = 20k mid window and the m = 100k window
O=gpurun_out/${1:-r6u}; mkdir -p $O
B=profiles/r06_blocks20k_basis_it61912.npz
for ga in 8192 2048 32768 1000000000; do
  for wd in 4096 2048 8192; do
    GK_SP_GA=$ga GK_SP_WIDE=$wd timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 --basis $B 200 20 > $O/w20_ga${ga}_wd${wd}.json 2>/dev/null || exit 1
  done
done
for ga in 8192 2048 32768; do
  GK_SP_GA=$ga timeout -k 10 120 python3 -u tools/sparse_window.py --it 500 > $O/w100_ga${ga}.json 2>/dev/null || exit 2
done
echo ok
