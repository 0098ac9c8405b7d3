#!/bin/bash
# next-call phase-I evaluation at the end of it_lim calls; init without zero-fills:
# LP tests (C3 full-size and bench-window parity), then the bench
set -e
mkdir -p gpurun_out/r03r
timeout -k 10 600 python -u -m pytest tests/test_gpu_lp.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r/lp_tests.log 2>&1
GK_INIT_LOG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-extra > gpurun_out/r03r/bench.json 2> gpurun_out/r03r/bench.err
echo ok
