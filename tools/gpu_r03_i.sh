#!/bin/bash
# Re-entry check of the final tree: the whole GPU suite (the driver's
# round-end command), smoke, then the driver's bench command
set -e
mkdir -p gpurun_out/r03i
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03i/tests.log 2>&1
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r03i/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r03i/bench.json 2> gpurun_out/r03i/bench.err
echo ok
