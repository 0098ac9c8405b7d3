# round 6: sparse window with the block-split ratio / pick scans, then the
# whole GPU suite and smoke() on the tree
O=gpurun_out/${1:-r6h}; mkdir -p $O
timeout -k 10 300 python3 -u tools/sparse_window.py --it 1000 > $O/win100k.json 2> $O/win100k.err || exit 1
timeout -k 10 300 python3 -u tools/sparse_window.py --it 2000 100 100 > $O/win20k.json 2> $O/win20k.err || exit 2
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc $?" >> $O/smoke.log
bash tools/prof_sparse_window.sh r6h_spw --it 1000 > $O/spw.log 2>&1; echo "spw rc $?" >> $O/spw.log
