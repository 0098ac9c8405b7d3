# round 6: node kernel vs engine mode on the fixtures with the largest count ratios
O=gpurun_out/${1:-r6p}; mkdir -p $O
timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 mixbig4 mixint11 c5s_12x32 > $O/default.json 2> $O/default.err || exit 1
GK_BNB_ENGINE_BYTES=0 timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 mixbig4 mixint11 > $O/engine.json 2> $O/engine.err || exit 2
echo ok
