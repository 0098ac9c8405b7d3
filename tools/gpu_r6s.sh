# round 6: the whole GPU suite, smoke() and the default bench on the tree
O=gpurun_out/${1:-r6s}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench rc $?" >> $O/bench.err
