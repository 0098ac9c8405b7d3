#!/bin/bash
# B&B pre-incumbent batch cap at its default: the whole GPU suite (the
# driver's round-end command), then the two B&B legs
set -e
mkdir -p gpurun_out/r03g
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g/tests.log 2>&1
for nm in gap c5s_12x30; do
  GK_BNB_LOG=1 timeout -k 10 120 python3 tools/prof_bnb.py $nm > gpurun_out/r03g/bnb_${nm}.log 2>&1
done
echo ok
