# round 6: A/B of the pipelined inv(M) loads (HEAD library in glpk.js_amd/ab_head.so)
set -e
O=gpurun_out/${1:-r6y}; mkdir -p $O
B=profiles/r06_blocks20k_basis_it61912.npz
for v in new old new2 old2; do
  case $v in old*) export GK_LIB_PATH=$GRAFT_REPO_ROOT/glpk.js_amd/ab_head.so;; *) unset GK_LIB_PATH;; esac
  timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 --basis $B 200 20 > $O/w20_$v.json 2>/dev/null
  timeout -k 10 120 python3 -u tools/sparse_window.py --it 1000 > $O/w100_$v.json 2>/dev/null
done
unset GK_LIB_PATH
bash tools/prof_sparse_window.sh r6y_new --it 1000 --basis $B 200 20 > $O/pn.log 2>&1
GK_LIB_PATH=$GRAFT_REPO_ROOT/glpk.js_amd/ab_head.so bash tools/prof_sparse_window.sh r6y_old --it 1000 --basis $B 200 20 > $O/po.log 2>&1
echo ok
