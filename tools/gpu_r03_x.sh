#!/bin/bash
# B&B batch processing on host workers: MIP tests (Python and JS, incl. the
# sharded runs), the B&B timing split; then the round profile of the final
# pivot kernels (tools/profile_round.sh r03)
set -e
mkdir -p gpurun_out/r03x
timeout -k 10 600 python -u -m pytest tests/test_gpu_mip.py tests/test_js.py tests/test_comm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x/mip_tests.log 2>&1
for nm in gap c5s_12x30; do
  GK_BNB_LOG=1 timeout -k 10 120 python3 tools/prof_bnb.py $nm > gpurun_out/r03x/bnb_${nm}.log 2>&1
  GK_BNB_THREADS=0 GK_BNB_LOG=1 timeout -k 10 120 python3 tools/prof_bnb.py $nm > gpurun_out/r03x/bnb_${nm}_serial.log 2>&1
done
timeout -k 10 1500 bash tools/profile_round.sh r03 > gpurun_out/profile_round_r03.log 2>&1
echo ok
