#!/bin/bash
# End of round 3 (Newton refinement on the tree): the refinement tests and the
# mid-solve window stats, the whole GPU suite, the driver's bench command and
# smoke.  Every GPU step has its own time limit; the first failure ends it.
set -e
R="$PWD"
O="$R/gpurun_out/r03f"
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_newton.py \
    tests/test_gpu_factor.py > "$O/tests_newton.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_mid -o mid -- \
    python3 -u tools/c3_mid.py 100000 30 > "$O/mid_newton.log" 2> "$O/mid_newton.err"
python3 tools/prof_stats.py /tmp/prof_mid/mid_results.db --marked --csv "$O/mid_window_stats.csv" > "$O/mid_window_stats.txt"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gputests.log" 2>&1
timeout -k 10 900 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python -u __graft_entry__.py smoke > "$O/smoke.log" 2>&1
echo ok
