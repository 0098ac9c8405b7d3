# round 6: colpass 8 segments in flight + GK_SP_SEG_MIN 4096 — tests, shard
# sim profile, the m = 20,020 full solve and mid window
set -e
O=gpurun_out/${1:-r6m}; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_lp_shard.py tests/test_gpu_sparse.py tests/test_sparse_factor.py tests/test_gpu_lp.py -m gpu > $O/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_ssim -o ssim -- python3 -u tools/shard_sim_prof.py 4 20000 5 > $O/sim.json 2> $O/sim.err
python3 tools/prof_stats.py /tmp/prof_ssim/ssim_results.db --marked --window 0 --csv $O/g1.csv > $O/g1.txt
python3 tools/prof_stats.py /tmp/prof_ssim/ssim_results.db --marked --window 1 --csv $O/g4.csv > $O/g4.txt
timeout -k 10 200 python3 -u tools/sparse_window.py --it 2000 --basis profiles/r06_blocks20k_basis_it61912.npz 200 20 > $O/win20k_mid.json 2> $O/win20k_mid.err
timeout -k 10 200 python3 -u tools/sparse_big.py --sparse blocks 200 20 > $O/full20k.json 2> $O/full20k.err
timeout -k 10 200 python3 -u tools/sparse_big.py blocks 40 5 > $O/blocks40.json 2> $O/blocks40.err
echo ok
