#!/bin/bash
# Newton refinement threshold: the first 40,000 pivots of the C3 dual (the
# structural block grows from 0 to ~2000) with the refinement from k >= 0
# (off), 1024 (default), 256 and 64; re-inversion time of the advance
set -e
R="$PWD"
O="$R/gpurun_out/r03thr"
mkdir -p "$O"
for K in 0 1024 256 64; do
    GK_NEWTON_MIN_K=$K timeout -k 10 200 python -u tools/c3_mid.py 40000 5 > "$O/thr_$K.log" 2>&1
done
echo ok
