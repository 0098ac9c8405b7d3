# round 6: the whole GPU suite and smoke() on HEAD
O=gpurun_out/${1:-r6f}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke rc $?" >> $O/smoke.log
