# round 6 diagnostics: the opt-in concurrent engine mode with the batch
# graphs off (GK_NO_GRAPH=1), three runs, against graphs on
O=gpurun_out/${1:-r6al}; mkdir -p $O
for r in 1 2 3; do
  GK_NO_GRAPH=1 GK_BNB_ENGINE_CONCURRENT=1 timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/nograph_$r.json 2>/dev/null || exit 1
  GK_BNB_ENGINE_CONCURRENT=1 timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/graph_$r.json 2>/dev/null || exit 2
done
GK_NO_GRAPH=1 timeout -k 10 200 python3 -u tools/bnb_time.py sparsebig1 > $O/nograph_seq.json 2>/dev/null || exit 3
echo ok
