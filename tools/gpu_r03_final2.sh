#!/bin/bash
# the driver's bench command and smoke on the final tree (Newton from k >= 512)
set -e
R="$PWD"
O="$R/gpurun_out/r03f2"
mkdir -p "$O"
timeout -k 10 900 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python -u __graft_entry__.py smoke > "$O/smoke.log" 2>&1
echo ok
