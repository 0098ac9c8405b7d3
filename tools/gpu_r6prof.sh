# round 6: the round profile (kernel stats, PMC traffic) and the default bench line
set -e
bash tools/profile_round.sh r06 > gpurun_out/r06_prof.log 2>&1
mkdir -p gpurun_out/r06
timeout -k 10 900 python3 -u bench.py > gpurun_out/r06/bench_default.json 2> gpurun_out/r06/bench_default.err
echo ok
