#!/bin/bash
# Round profile on one MI355X (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats of the bench command the driver runs
#      (--gpus 1 --steps 20 --warmup 5; the CPU baseline and the extra
#      configurations, which run after the timed region, are left out: their
#      traces exceed what gpurun copies back) -> rNN/stats*.csv/json and the
#      bench line of that run (prof_bench.json)
#   2. two --pmc passes of the same command (FETCH_SIZE, WRITE_SIZE; separate
#      runs, no traces), timed region only   -> rNN/pmc_traffic.json
#   3. the command and commit profiled        -> rNN/profile_meta.json
# bench.py reads these (copied to profiles/) only when the profiled command
# matches its own arguments.  Raw traces stay in /tmp on the box; every GPU
# step has its own time limit and the script stops at the first failure.
set -e
R=${1:-r03}
OUT=gpurun_out/$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=/tmp/prof_$R
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $T/prof -o run -- python3 bench.py $ARGS > $OUT/prof_bench.json 2> $OUT/prof.err
python3 tools/prof_stats.py $T/prof/run_results.db --csv $OUT/stats.csv > $OUT/stats_grid.txt
python3 tools/prof_stats.py $T/prof/run_results.db --marked --csv $OUT/stats_timed.csv --json $OUT/stats_timed.json > /dev/null
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $T/pmc_fetch -o run -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $T/pmc_write -o run -- python3 bench.py $ARGS > /dev/null 2> $OUT/pmc_write.err
python3 tools/pmc_traffic.py $T/pmc_fetch $T/pmc_write $OUT/pmc_traffic.json --marked > /dev/null
python3 - "$OUT" "$ARGS" <<'EOF'
import json, subprocess, sys
out, args = sys.argv[1], sys.argv[2]
head = open(".git_head").read().strip() if __import__("os").path.exists(".git_head") else None
a = args.split()
val = lambda k, d: int(a[a.index(k) + 1]) if k in a else d
meta = {"cmd": "python3 bench.py " + args, "head": head,
        "args": {"steps": val("--steps", 20), "warmup": val("--warmup", 5), "pivots_per_step": 100,
                 "m": 4096, "n": 16384}}
json.dump(meta, open(out + "/profile_meta.json", "w"), indent=1)
EOF
echo done
