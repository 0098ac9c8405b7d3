#!/bin/bash
# kernel-trace stats of the bench's timed region (no PMC), plus a bench line
set -e
mkdir -p gpurun_out/r03d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p3d -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra > gpurun_out/r03d/prof_bench.json 2> gpurun_out/r03d/prof.err
python3 tools/prof_stats.py /tmp/p3d/run_results.db --marked --csv gpurun_out/r03d/stats_timed.csv --json gpurun_out/r03d/stats_timed.json > /dev/null
timeout -k 10 300 python3 bench.py --no-cpu --no-extra > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err
timeout -k 10 300 python3 bench.py --no-cpu --no-extra > gpurun_out/r03d/bench2.json 2>> gpurun_out/r03d/bench.err
echo ok
