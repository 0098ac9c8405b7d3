# round 6: m = 20,020 mid-solve basis (12 s into the solve), then a 2,000-pivot
# window from it plain and under rocprofv3 --kernel-trace --stats
set -e
O=gpurun_out/${1:-r6j}; mkdir -p $O
timeout -k 10 120 python3 -u tools/sparse_big.py --sparse --tm 12 --save $O/b20k_mid.npz blocks 200 20 > $O/mid.json 2> $O/mid.err
bash tools/prof_sparse_window.sh r6j_spw --it 2000 --basis $O/b20k_mid.npz 200 20 > $O/spw.log 2>&1
echo ok
