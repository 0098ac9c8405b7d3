# round 6 diagnostics: engine-mode node counts with new device memory
# poisoned (GK_DEBUG_POISON), one node LP at a time and concurrent
O=gpurun_out/${1:-r6af}; mkdir -p $O
for pz in none 0 0xff 0x7f; do
  if [ $pz = none ]; then unset GK_DEBUG_POISON; else export GK_DEBUG_POISON=$pz; fi
  timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/seq_$pz.json 2> $O/seq_$pz.err || exit 1
  GK_BNB_ENGINE_CONCURRENT=1 timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/conc_$pz.json 2> $O/conc_$pz.err || exit 2
done
unset GK_DEBUG_POISON
for r in 1 2; do GK_BNB_ENGINE_CONCURRENT=1 timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/conc_rep$r.json 2>/dev/null || exit 3; done
echo ok
