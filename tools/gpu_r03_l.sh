#!/bin/bash
# instruction-fetch microbenchmark (s_nop bodies)
set -e
mkdir -p gpurun_out/r03l
hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_icache tools/ubench_icache.hip 2>/dev/null
timeout -k 10 60 /tmp/ubench_icache > gpurun_out/r03l/icache.txt 2>&1
echo ok
