#!/bin/bash
# Newton refinement, second pass: tests, then the C3 mid-solve window under
# the kernel trace (GEMM durations; the trace stays in /tmp, only the stats
# come back), and the Gauss-Jordan-only run beside it
set -e
R="$PWD"
mkdir -p "$R/gpurun_out/r03z2"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_newton.py \
    > "$R/gpurun_out/r03z2/tests_newton.log" 2>&1
GK_DRIFT_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_mid -o mid -- \
    python3 -u tools/c3_mid.py 100000 30 > "$R/gpurun_out/r03z2/mid_newton.log" 2> "$R/gpurun_out/r03z2/mid_newton.err"
find /tmp/prof_mid -name '*kernel_stats.csv' -exec cp {} "$R/gpurun_out/r03z2/" \;
GK_DRIFT_LOG=1 GK_NEWTON_MIN_K=0 timeout -k 10 300 python -u tools/c3_mid.py 100000 30 > "$R/gpurun_out/r03z2/mid_gj.log" \
    2> "$R/gpurun_out/r03z2/mid_gj.err"
echo ok
