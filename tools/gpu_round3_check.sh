#!/bin/bash
# One GPU call: the whole GPU suite, the B&B timing split, and the
# re-inversion at k = 4096 with the look-ahead under rocprofv3 (the process
# must exit cleanly: the look-ahead streams are owned by the context now).
# Every GPU step has its own time limit; the script stops at the first
# failing step.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
GK_BNB_LOG=1 timeout -k 10 200 python tools/prof_bnb.py gap > gpurun_out/bnb_gap.log 2>&1
GK_BNB_LOG=1 timeout -k 10 200 python tools/prof_bnb.py c5s_12x30 > gpurun_out/bnb_c5s.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prein -o run -- python3 tools/prof_reinvert.py 4096 4096 2 > gpurun_out/reinv_la.log 2>&1
echo "reinv rc=$?" >> gpurun_out/reinv_la.log
python3 tools/prof_stats.py /tmp/prein/run_results.db --csv gpurun_out/reinv_la_stats.csv > gpurun_out/reinv_la_grid.txt
