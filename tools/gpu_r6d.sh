# round 6: the whole GPU suite on HEAD, the B&B legs (engine mode on the
# m = 320 ... 800 fixtures), then the node-selection variants on gap / C5s
O=gpurun_out/${1:-r6d}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 sparsebig2 sparsebig3 sparsebig4 > $O/bnb.json 2> $O/bnb.err || exit 2
for v in "GK_BNB_BLB_WINDOW=0" "GK_BNB_BLB_WINDOW=4096" "GK_BNB_WINBATCH=8" "GK_BNB_WINBATCH=32" "GK_BNB_WINBATCH=8 GK_BNB_DEPTH=1"; do
  echo "== $v" >> $O/sel.json
  env $v timeout -k 10 200 python3 -u tools/bnb_time.py gap c5s_12x30 c5s_12x40 >> $O/sel.json 2>> $O/sel.err || exit 3
done
