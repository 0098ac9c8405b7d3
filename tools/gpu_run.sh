#!/bin/bash
# One GPU session through gpurun, from the repo root:
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_run.sh NAME STEP [STEP ...]
# Output goes to gpurun_out/NAME/.  Every step runs under its own time limit
# and the script stops at the first failure (set -e), so nothing more touches
# the GPU after a fault, an abort or a timeout.  Steps:
#   tests            the whole -m gpu suite (the driver's round-end command)
#   tests:F1,F2      -m gpu tests of the named files (tests/F1 ...)
#   k:EXPR           -m gpu tests selected by -k EXPR
#   smoke            __graft_entry__.py smoke
#   bench            python bench.py (defaults: the driver's command)
#   bench:ARGS       python bench.py ARGS (commas for spaces)
#   profile          tools/profile_round.sh (rocprofv3 stats + PMC passes)
#   apitrace         rocprofv3 HIP API + kernel + copy traces (CSV) of a short bench
#   ktrace           rocprofv3 kernel trace of the bench's timed region: stats
#                    and the idle gaps between consecutive kernels
#   py:SCRIPT,ARGS   python3 -u SCRIPT ARGS (tools/…; commas for spaces) -> SCRIPT.<k>.log / .err
#   pytSECS:SCRIPT,ARGS  the same under a limit of SECS seconds (default 900)
set -e
NAME=$1; shift
O="$PWD/gpurun_out/$NAME"
mkdir -p "$O"
export TMPDIR=/tmp
k=0
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
for step in "$@"; do
    case "$step" in
        tests) timeout -k 10 900 $PYT tests > "$O/tests.log" 2>&1 ;;
        tests:*) f=${step#tests:}; timeout -k 10 900 $PYT $(echo "$f" | tr ',' '\n' | sed 's|^|tests/|') \
                     > "$O/tests_$(echo "$f" | tr ',/' '__').log" 2>&1 ;;
        k:*) timeout -k 10 900 $PYT tests -k "${step#k:}" > "$O/tests_k.log" 2>&1 ;;
        smoke) timeout -k 10 300 python -u __graft_entry__.py smoke > "$O/smoke.log" 2>&1 ;;
        bench) timeout -k 10 900 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" ;;
        bench:*) a=$(echo "${step#bench:}" | tr ',' ' ');
                 timeout -k 10 900 python -u bench.py $a > "$O/bench_args.json" 2> "$O/bench_args.err" ;;
        profile) bash tools/profile_round.sh "$NAME/profile" ;;
        apitrace) cd /tmp && cd "$GRAFT_REPO_ROOT";
                timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv \
                    -d /tmp/at_$NAME -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 2 --no-cpu --no-extra \
                    > "$O/at_bench.json" 2> "$O/at.err";
                mkdir -p "$O/apitrace"; find /tmp/at_$NAME -name '*.csv' -exec cp {} "$O/apitrace/" \; ;;
        ktrace) cd /tmp && cd "$GRAFT_REPO_ROOT";
                timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_$NAME -o run -- python3 bench.py \
                    --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra > "$O/kt_bench.json" 2> "$O/kt.err";
                python3 tools/prof_stats.py /tmp/kt_$NAME/run_results.db --marked --csv "$O/kt_stats.csv" \
                    --gaps "$O/kt_gaps.txt" > "$O/kt_grid.txt" ;;
        py:*) a=$(echo "${step#py:}" | tr ',' ' '); s=$(basename ${a%% *} .py); k=$((k + 1));
              timeout -k 10 900 python3 -u $a > "$O/$s.$k.log" 2> "$O/$s.$k.err" ;;
        pyt*:*) lim=${step%%:*}; lim=${lim#pyt}; a=$(echo "${step#*:}" | tr ',' ' '); s=$(basename ${a%% *} .py);
              k=$((k + 1)); timeout -k 10 "$lim" python3 -u $a > "$O/$s.$k.log" 2> "$O/$s.$k.err" ;;
        rprof:*) a=$(echo "${step#rprof:}" | tr ',' ' '); s=$(basename ${a%% *} .py); k=$((k + 1));
              cd /tmp && cd "$GRAFT_REPO_ROOT";
              timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/rp_${NAME}_$k -o run -- python3 -u $a \
                  > "$O/rp_$s.$k.log" 2> "$O/rp_$s.$k.err";
              python3 tools/prof_stats.py /tmp/rp_${NAME}_$k/run_results.db --csv "$O/rp_$s.$k.csv" --gaps "$O/rp_$s.$k.gaps" \
                  > "$O/rp_$s.$k.txt" ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
    echo "step $step ok"
done
echo done
