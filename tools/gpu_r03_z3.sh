#!/bin/bash
# Newton refinement, third pass: GEMM kernel durations in the C3 mid-solve
# window (stats of the marked window only), then the C3 full dual solve with
# the refinement (default) and with Gauss-Jordan only
set -e
R="$PWD"
O="$R/gpurun_out/r03z3"
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_mid -o mid -- \
    python3 -u tools/c3_mid.py 100000 30 > "$O/mid_newton.log" 2> "$O/mid_newton.err"
python3 tools/prof_stats.py /tmp/prof_mid/mid_results.db --marked --csv "$O/mid_window_stats.csv" > "$O/mid_window_stats.txt"
timeout -k 10 400 python -u tools/c3_full.py 4096 16384 3 300000 > "$O/full_newton.jsonl" 2> "$O/full_newton.err"
GK_NEWTON_MIN_K=0 timeout -k 10 400 python -u tools/c3_full.py 4096 16384 3 300000 > "$O/full_gj.jsonl" 2> "$O/full_gj.err"
echo ok
