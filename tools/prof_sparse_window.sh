#!/bin/bash
# The sparse factor's pivot window (tools/sparse_window.py) plain and under
# rocprofv3 --kernel-trace --stats (timed window only): gpurun_out/$1/
set -e
O="$PWD/gpurun_out/${1:-spw}"
shift || true
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/sparse_window.py "$@" > "$O/window.json" 2> "$O/window.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_spw -o spw -- python3 -u tools/sparse_window.py "$@" \
    > "$O/window_prof.json" 2> "$O/window_prof.err"
python3 tools/prof_stats.py /tmp/prof_spw/spw_results.db --marked --csv "$O/stats_timed.csv" > "$O/stats_timed.txt"
echo ok
