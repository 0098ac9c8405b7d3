#!/bin/bash
# C3 full dual solve on the final tree (Newton from k >= 512) and with the
# refinement from k >= 64
set -e
R="$PWD"
O="$R/gpurun_out/r03full2"
mkdir -p "$O"
timeout -k 10 400 python -u tools/c3_full.py 4096 16384 3 300000 > "$O/full_512.jsonl" 2> "$O/full_512.err"
GK_NEWTON_MIN_K=64 timeout -k 10 400 python -u tools/c3_full.py 4096 16384 3 300000 > "$O/full_64.jsonl" 2> "$O/full_64.err"
echo ok
