set -e
O=gpurun_out/paths
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/prof_paths.py > $O/plain.jsonl 2> $O/plain.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/prof_paths.py > $O/prof.jsonl 2> $O/prof.err
for w in 0 1 2 3; do python3 tools/prof_stats.py $O/prof/run_results.db --marked --window $w --csv $O/w$w.csv > $O/w$w.txt; done
echo done
