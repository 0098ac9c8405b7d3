#!/bin/bash
# Round-3 GPU step (run through gpurun from the repo root): parity tests of
# the factorization parameters and the LP paths, a short bench, then the round
# profile (tools/profile_round.sh) and the graph-replay pivot trace.
set -e
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_bfcp.py tests/test_presolve.py tests/test_gpu_lp.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r03/tests_lp.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-extra > gpurun_out/r03/bench_quick.json 2> gpurun_out/r03/bench_quick.err
bash tools/profile_round.sh r03
GK_TRACE_GRAPH=1 timeout -k 10 200 python3 tools/trace_pivot.py 4096 16384 1000 > gpurun_out/r03/trace_pivot_graph.txt 2>&1
echo ok
