O=gpurun_out/${1:-r6e}; mkdir -p $O
timeout -k 10 170 python3 -u tools/bnb_time.py sparsebig2 sparsebig3 > $O/bnb23.json 2> $O/bnb.err || exit 2
timeout -k 10 170 python3 -u tools/bnb_time.py sparsebig4 > $O/bnb4.json 2>> $O/bnb.err
timeout -k 10 170 python3 -u tools/bnb_time.py gap c5s_12x30 c5s_12x40 > $O/sel_default.json 2>> $O/bnb.err
GK_BNB_BLB_WINDOW=0 timeout -k 10 170 python3 -u tools/bnb_time.py gap c5s_12x30 c5s_12x40 > $O/sel_nowin.json 2>> $O/bnb.err
GK_BNB_WINBATCH=8 timeout -k 10 170 python3 -u tools/bnb_time.py gap c5s_12x30 c5s_12x40 > $O/sel_wb8.json 2>> $O/bnb.err
