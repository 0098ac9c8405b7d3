# round 6: column pass segments in flight A/B under the simulated 4-rank profile
set -e
O=gpurun_out/${1:-r6n}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ssim -o ssim -- python3 -u tools/shard_sim_prof.py 4 20000 5 > $O/sim.json 2> $O/sim.err
python3 tools/prof_stats.py /tmp/prof_ssim/ssim_results.db --marked --window 0 --csv $O/g1.csv > $O/g1.txt
python3 tools/prof_stats.py /tmp/prof_ssim/ssim_results.db --marked --window 1 --csv $O/g4.csv > $O/g4.txt
timeout -k 10 300 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_lp_shard.py -m gpu > $O/tests.log 2>&1
echo ok
