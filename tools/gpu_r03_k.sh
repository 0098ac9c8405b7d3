#!/bin/bash
# instruction-fetch microbenchmark; C3 advance to 100k with the drift log
set -e
mkdir -p gpurun_out/r03k
hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_icache tools/ubench_icache.hip 2>/dev/null
timeout -k 10 60 /tmp/ubench_icache > gpurun_out/r03k/icache.txt 2>&1
GK_DRIFT_LOG=1 timeout -k 10 300 python3 -u tools/instab_probe.py 100000 > gpurun_out/r03k/drift.log 2>&1
echo ok
