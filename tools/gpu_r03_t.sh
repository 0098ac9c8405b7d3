#!/bin/bash
# k_dual_update's three LDS sums in separate waves: LP parity tests, then A/B
# on one box (ab/libA.so = the previous combine)
set -e
mkdir -p gpurun_out/r03t
timeout -k 10 600 python -u -m pytest tests/test_gpu_lp.py tests/test_panel.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03t/lp_tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-extra > gpurun_out/r03t/B_$r.json 2> gpurun_out/r03t/B_$r.err
  GK_LIB_PATH=$PWD/ab/libA.so timeout -k 10 300 python -u bench.py --no-cpu --no-extra > gpurun_out/r03t/A_$r.json 2> gpurun_out/r03t/A_$r.err
done
echo ok
