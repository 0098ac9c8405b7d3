#!/bin/bash
# position-array change: LP / MIP / C3 GPU parity, PMC traffic of the pivot
# kernels, then the bench
set -e
mkdir -p gpurun_out/r03e
timeout -k 10 900 python -u -m pytest tests/test_gpu_lp.py tests/test_bfcp.py tests/test_gpu_mip.py tests/test_presolve.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-extra > gpurun_out/r03e/bench.json 2> gpurun_out/r03e/bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p3e -o run -- python3 bench.py $ARGS > gpurun_out/r03e/prof_bench.json 2> gpurun_out/r03e/prof.err
python3 tools/prof_stats.py /tmp/p3e/run_results.db --marked --csv gpurun_out/r03e/stats_timed.csv --json gpurun_out/r03e/stats_timed.json > /dev/null
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/p3e_f -o run -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/r03e/pmc_fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/p3e_w -o run -- python3 bench.py $ARGS > /dev/null 2> gpurun_out/r03e/pmc_write.err
python3 tools/pmc_traffic.py /tmp/p3e_f /tmp/p3e_w gpurun_out/r03e/pmc_traffic.json --marked > /dev/null
echo ok
