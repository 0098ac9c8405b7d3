#!/bin/bash
# re-inversion k=4096 under rocprofv3 (per-kernel durations)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03q
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prein -o run -- python3 tools/prof_reinvert.py 4096 4096 2 > gpurun_out/r03q/reinv.log 2>&1
python3 tools/prof_stats.py /tmp/prein/run_results.db --csv gpurun_out/r03q/reinv_stats.csv > gpurun_out/r03q/reinv_grid.txt
echo ok
