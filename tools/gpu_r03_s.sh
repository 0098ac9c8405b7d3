#!/bin/bash
# A/B on one box: the next-call phase-I evaluation on / off (GK_NEXT_AUX=0)
set -e
mkdir -p gpurun_out/r03s
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-extra > gpurun_out/r03s/on_$r.json 2> gpurun_out/r03s/on_$r.err
  GK_NEXT_AUX=0 timeout -k 10 300 python -u bench.py --no-cpu --no-extra > gpurun_out/r03s/off_$r.json 2> gpurun_out/r03s/off_$r.err
done
echo ok
