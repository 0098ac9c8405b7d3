#!/bin/bash
# B&B batch cap before the first incumbent: gap and C5s 12x30 at several caps
set -e
mkdir -p gpurun_out/r03f
for cap in 0 8 16 32 64 128; do
  for nm in gap c5s_12x30; do
    GK_BNB_PRECAP=$cap GK_BNB_LOG=1 timeout -k 10 120 python3 tools/prof_bnb.py $nm > gpurun_out/r03f/bnb_${nm}_${cap}.log 2>&1
  done
done
echo ok
