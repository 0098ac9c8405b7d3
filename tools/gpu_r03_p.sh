#!/bin/bash
# unrolled Gauss-Jordan panel steps: factor tests, re-inversion device time
set -e
mkdir -p gpurun_out/r03p
timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03p/factor_tests.log 2>&1
for k in 2048 4096; do
  GK_GJ_TIME=1 timeout -k 10 120 python3 -u tools/prof_reinvert.py $k $k 3 > gpurun_out/r03p/reinv_$k.log 2>&1
done
GK_INIT_LOG=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu --no-extra > gpurun_out/r03p/bench.json 2> gpurun_out/r03p/bench.err
echo ok
