# rocprof kernel statistics of the first seconds of the m = 20,020 sparse dual solve
O=gpurun_out/${1:-s20kp}
mkdir -p $O/raw
cd $O/raw && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d . -o s20k -- python3 -u ../../../tools/sparse_big.py --tm 6 blocks 200 20 > ../run.json 2> ../run.err
e=$?
cp $(find . -name "*kernel_stats.csv" | head -1) ../kernel_stats.csv 2>/dev/null
cd .. && rm -rf raw
exit $e
