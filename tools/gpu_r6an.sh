# round 6: the whole GPU suite on the final tree
O=gpurun_out/${1:-r6an}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
