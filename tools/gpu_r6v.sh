# round 6: sparse plan knobs, second sweep, and the m = 20,020 full solve
# with the candidate setting
O=gpurun_out/${1:-r6v}; mkdir -p $O
B=profiles/r06_blocks20k_basis_it61912.npz
for ga in 2048 1024 512; do
  for wd in 2048 1024 512; do
    GK_SP_GA=$ga GK_SP_WIDE=$wd timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 --basis $B 200 20 > $O/w20_ga${ga}_wd${wd}.json 2>/dev/null || exit 1
  done
done
for wd in 4096 2048 1024; do
  GK_SP_GA=2048 GK_SP_WIDE=$wd timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 > $O/w100_ga2048_wd${wd}.json 2>/dev/null || exit 2
done
timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 > $O/w100_default.json 2>/dev/null || exit 3
GK_SP_GA=2048 GK_SP_WIDE=2048 timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/full20k_ga2048_wd2048.json 2> $O/full20k.err || exit 4
echo ok
