# round 6: the whole GPU suite on HEAD, then the B&B legs (engine mode on the
# m = 320 ... 800 fixtures)
O=gpurun_out/${1:-r6d}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1
echo "tests rc $?" >> $O/tests.log
timeout -k 10 300 python3 -u tools/bnb_time.py sparsebig1 sparsebig2 sparsebig3 sparsebig4 > $O/bnb.json 2> $O/bnb.err || exit 2
