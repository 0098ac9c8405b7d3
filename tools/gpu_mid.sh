# C3 mid-solve window (pivots 100,000-103,000): rate, then rocprof kernel statistics of the window
O=gpurun_out/${1:-mid}
mkdir -p $O
timeout -k 10 200 python3 -u tools/c3_mid.py 100000 30 > $O/mid.txt 2>&1 || exit 2
tail -1 $O/mid.txt
mkdir -p $O/raw && cd $O/raw && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d . -o mid -- python3 -u ../../../tools/c3_mid.py 100000 30 > ../mid_prof.txt 2>&1 || exit 3
DB=$(find . -name "*.db" | head -1)
python3 ../../../tools/prof_stats.py $DB --marked > ../window_stats.txt || exit 4
cd .. && rm -rf raw
head -25 window_stats.txt
