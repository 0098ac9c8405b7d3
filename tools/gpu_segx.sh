O=gpurun_out/${1:-segx}
mkdir -p $O
for x in 0 1 2 3; do
  GK_SP_SEGX=$x GK_SP_STAMPS=$O/stamps_$x.txt timeout -k 10 200 python3 -u tools/sparse_window.py --it 200 > $O/run_$x.json 2>&1 || exit 1
  GK_SP_SEGX=$x timeout -k 10 200 python3 -u tools/sparse_window.py --it 1000 > $O/win_$x.json 2>&1 || exit 1
done
