#!/bin/bash
# whole GPU suite on the current tree, then the bench (default command) twice
set -e
mkdir -p gpurun_out/r03v
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03v/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-extra > gpurun_out/r03v/bench_$r.json 2> gpurun_out/r03v/bench_$r.err
done
for nm in gap c5s_12x30; do
  GK_BNB_LOG=1 timeout -k 10 120 python3 tools/prof_bnb.py $nm > gpurun_out/r03v/bnb_${nm}.log 2>&1
done
echo ok
