# rocprof kernel statistics of the blocks-40 sparse dual solve (m = 4,005)
O=gpurun_out/${1:-b40p}
mkdir -p $O/raw
cd $O/raw && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d . -o b40 -- python3 -u ../../../tools/sparse_big.py blocks 40 5 > ../run.json 2> ../run.err
e=$?
cp $(find . -name "*kernel_stats.csv" | head -1) ../kernel_stats.csv 2>/dev/null
cd .. && rm -rf raw
exit $e
