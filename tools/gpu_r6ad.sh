# round 6: engine-mode batch width (GK_BNB_ENGINE_BATCH) on the sparse MIPs
O=gpurun_out/${1:-r6ad}; mkdir -p $O
for b in 8 16 4; do
  GK_BNB_ENGINE_BATCH=$b timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 sparsebig2 sparsebig3 sparsebig4 > $O/b$b.json 2> $O/b$b.err || exit 1
done
echo ok
