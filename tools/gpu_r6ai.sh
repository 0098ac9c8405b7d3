# round 6 diagnostics: concurrent engine mode with one worker (the batch-start
# cutoff, a separate context, no concurrency) against eight workers
O=gpurun_out/${1:-r6ai}; mkdir -p $O
for r in 1 2 3; do
  GK_BNB_ENGINE_CONCURRENT=1 GK_BNB_ENGINE_WORKERS=1 timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/w1_$r.json 2>/dev/null || exit 1
  GK_BNB_ENGINE_CONCURRENT=1 timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/w8_$r.json 2>/dev/null || exit 2
done
echo ok
