#!/bin/bash
# the driver's bench command on the final tree (CPU baseline and extras on),
# then smoke
set -e
mkdir -p gpurun_out/r03y
timeout -k 10 900 python -u bench.py > gpurun_out/r03y/bench.json 2> gpurun_out/r03y/bench.err
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r03y/smoke.log 2>&1
echo ok
