set -e
mkdir -p gpurun_out/r5d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--gpus 1 --steps 20 --warmup 5 --no-cpu --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pn -o run -- python3 bench.py $ARGS > gpurun_out/r5d/new.json 2> /dev/null
python3 tools/prof_stats.py /tmp/pn/run_results.db --marked --csv gpurun_out/r5d/new_timed.csv > gpurun_out/r5d/new_timed.txt
GK_LIB_PATH=ab/r04/libglpk_mi355x.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/po -o run -- python3 bench.py $ARGS > gpurun_out/r5d/old.json 2> /dev/null
python3 tools/prof_stats.py /tmp/po/run_results.db --marked --csv gpurun_out/r5d/old_timed.csv > gpurun_out/r5d/old_timed.txt
