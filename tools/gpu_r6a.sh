O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 400 python3 -u tools/bnb_time.py c5s_12x40 c5s_12x42 > $O/bnb.json 2> $O/bnb.err || exit 1
