# round 6 diagnostics: engine-mode node counts with a fresh factor per node
# LP (GK_BNB_FRESH_FB), twice, against the default
O=gpurun_out/${1:-r6ah}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/default_$r.json 2>/dev/null || exit 1
  GK_BNB_FRESH_FB=1 timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 > $O/fresh_$r.json 2>/dev/null || exit 2
done
echo ok
