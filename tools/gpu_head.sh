# graph head A/B on the headline bench (no extras) and the call timeline
O=gpurun_out/${1:-head}
mkdir -p $O
for h in 8 0 8 0; do GK_GRAPH_HEAD=$h timeout -k 10 200 python3 -u bench.py --no-extra --no-cpu >> $O/bench_h$h.json 2>> $O/bench.err || exit 1; done
timeout -k 10 120 python3 -u tools/call_log.py 5 5 > $O/calls.txt 2>&1 || exit 2
