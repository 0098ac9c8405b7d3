# round 6: the m = 20,020 mid-solve window (pivot 61,912) by the step count
# from which a sweep is segmented (GK_SP_SEG_MIN), and its level histograms
O=gpurun_out/${1:-r6l}; mkdir -p $O
B=profiles/r06_blocks20k_basis_it61912.npz
GK_SP_LEVELS=1 timeout -k 10 200 python3 -u tools/sparse_window.py --it 20 --basis $B 200 20 > $O/levels.json 2> $O/levels.txt || exit 1
for v in 16384 8192 4096 2048; do
  GK_SP_SEG_MIN=$v timeout -k 10 200 python3 -u tools/sparse_window.py --it 2000 --basis $B 200 20 > $O/win_seg$v.json 2> $O/win_seg$v.err || exit 2
done
echo ok
