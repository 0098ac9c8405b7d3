#!/bin/bash
set -e
O="$PWD/gpurun_out/r04g"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GK_SPARSE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_sp -o sp -- python3 -u tools/sparse_big.py --sparse blocks 40 > "$O/sp.log" 2> "$O/sp.err"
python3 tools/prof_stats.py /tmp/prof_sp/sp_results.db --csv "$O/stats.csv" > "$O/stats.txt"
echo ok
