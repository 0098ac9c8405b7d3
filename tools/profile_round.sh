#!/bin/bash
# Round profile on one MI355X (run through gpurun from the repo root):
#   1. the default bench line            -> gpurun_out/rNN/bench.json
#   2. rocprofv3 --kernel-trace --stats of the headline bench (no extras:
#      their traces exceed what gpurun copies back) -> rNN/stats*.csv/json
#   3. two --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs, no traces)
#      of a short bench                  -> rNN/pmc_traffic.json
# Raw traces stay in /tmp on the box; every GPU step has its own time limit
# and the script stops at the first failure.
set -e
R=${1:-r01}
OUT=gpurun_out/$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=/tmp/prof_$R
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $T/prof -o run -- python3 bench.py --no-extra > $OUT/prof_bench.json 2> $OUT/prof.err
python3 tools/prof_stats.py $T/prof/run_results.db --csv $OUT/stats.csv > $OUT/stats_grid.txt
python3 tools/prof_stats.py $T/prof/run_results.db --marked --csv $OUT/stats_timed.csv --json $OUT/stats_timed.json > /dev/null
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/pmc_fetch -o run -- python3 bench.py --no-cpu --no-extra > /dev/null 2> $OUT/pmc_fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/pmc_write -o run -- python3 bench.py --no-cpu --no-extra > /dev/null 2> $OUT/pmc_write.err
python3 tools/pmc_traffic.py $T/pmc_fetch $T/pmc_write $OUT/pmc_traffic.json --marked > /dev/null
echo done
