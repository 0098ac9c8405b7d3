#!/bin/bash
# Newton refinement of the scheduled re-inversion: GPU tests, the factor and
# LP suites it touches, and the C3 mid-solve window with and without it
set -e
mkdir -p gpurun_out/r03z
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_newton.py \
    tests/test_gpu_factor.py > gpurun_out/r03z/tests_newton.log 2>&1
timeout -k 10 300 python -u tools/c3_mid.py 100000 10 > gpurun_out/r03z/mid_newton.log 2>&1
GK_NEWTON_MIN_K=0 timeout -k 10 300 python -u tools/c3_mid.py 100000 10 > gpurun_out/r03z/mid_gj.log 2>&1
echo ok
