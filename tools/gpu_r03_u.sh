#!/bin/bash
# fused inner-panel schedule of the re-inversion: factor tests (incl. the
# fused / unfused bit-identity test), device time at k = 2048 / 4096 both ways
set -e
mkdir -p gpurun_out/r03u
timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u/factor_tests.log 2>&1
for k in 1024 2048 4096; do
  GK_GJ_TIME=1 timeout -k 10 120 python3 -u tools/prof_reinvert.py $k $k 3 > gpurun_out/r03u/fused_$k.log 2>&1
  GK_GJ_FUSED=0 GK_GJ_TIME=1 timeout -k 10 120 python3 -u tools/prof_reinvert.py $k $k 3 > gpurun_out/r03u/pairs_$k.log 2>&1
done
echo ok
