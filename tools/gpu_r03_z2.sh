#!/bin/bash
# Newton refinement, second pass: tests, then the C3 mid-solve window under
# the kernel trace (GEMM durations), and the Gauss-Jordan-only run beside it
set -e
mkdir -p gpurun_out/r03z2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_newton.py \
    > gpurun_out/r03z2/tests_newton.log 2>&1
GK_DRIFT_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03z2/prof -o mid -- \
    python3 -u tools/c3_mid.py 100000 30 > gpurun_out/r03z2/mid_newton.log 2> gpurun_out/r03z2/mid_newton.err
GK_DRIFT_LOG=1 GK_NEWTON_MIN_K=0 timeout -k 10 300 python -u tools/c3_mid.py 100000 30 > gpurun_out/r03z2/mid_gj.log \
    2> gpurun_out/r03z2/mid_gj.err
echo ok
