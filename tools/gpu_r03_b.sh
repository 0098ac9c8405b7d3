#!/bin/bash
# Round-3 GPU step B: LP / bfcp / presolve / JS GPU tests, then the full bench.
set -e
mkdir -p gpurun_out/r03b
timeout -k 10 900 python -u -m pytest tests/test_gpu_lp.py tests/test_bfcp.py tests/test_presolve.py tests/test_js.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b/tests.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err
echo ok
