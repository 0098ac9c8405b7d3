# round 6, final tree: the whole GPU suite, smoke(), the default bench, then
# the round profile (kernel stats and PMC traffic of the bench command)
bash tools/gpu_r6s.sh r6final || exit 1
bash tools/profile_round.sh r06 > gpurun_out/r06_prof_final.log 2>&1 || exit 2
echo ok
