#!/bin/bash
# Newton threshold 512 (new default): the first 40,000 C3 pivots, the
# refinement tests and the whole GPU suite
set -e
R="$PWD"
O="$R/gpurun_out/r03thr2"
mkdir -p "$O"
timeout -k 10 200 python -u tools/c3_mid.py 40000 5 > "$O/thr_512.log" 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gputests.log" 2>&1
echo ok
