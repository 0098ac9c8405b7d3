#!/bin/bash
# re-inversion at k = 4096 under rocprofv3 (tools/prof_reinvert.py), after the
# factor tests; optional environment variants (experiments) as arguments
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_factor.py -x -q --timeout 200 --timeout-method thread > gpurun_out/factor.log 2>&1
i=0
for v in "X=0" "$@"; do
  timeout -k 10 300 env $v rocprofv3 --kernel-trace --stats -d /tmp/prein$i -o run -- python3 tools/prof_reinvert.py 4096 4096 2 > gpurun_out/reinv$i.log 2>&1
  python3 tools/prof_stats.py /tmp/prein$i/run_results.db --csv gpurun_out/reinv_stats$i.csv > gpurun_out/reinv_grid$i.txt
  i=$((i+1))
done
