#!/bin/bash
# Newton refinement, fourth pass (update GEMM on the column-major copy): the
# refinement tests and the factor suite, then the mid-solve window stats
set -e
R="$PWD"
O="$R/gpurun_out/r03z4"
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_newton.py \
    tests/test_gpu_factor.py > "$O/tests_newton.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_mid -o mid -- \
    python3 -u tools/c3_mid.py 100000 30 > "$O/mid_newton.log" 2> "$O/mid_newton.err"
python3 tools/prof_stats.py /tmp/prof_mid/mid_results.db --marked --csv "$O/mid_window_stats.csv" > "$O/mid_window_stats.txt"
echo ok
