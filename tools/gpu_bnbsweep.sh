# B&B batch-shape sweep on the small trees (GK_BNB_CAP / GK_BNB_PRECAP / GK_BNB_DEPTH)
O=gpurun_out/${1:-bnbsweep}
mkdir -p $O
for cfg in "0 8 2" "64 8 2" "16 8 2" "8 8 2" "4 4 2" "8 8 1" "4 4 1" "2 2 1"; do
  set -- $cfg
  echo "cap $1 precap $2 depth $3" >> $O/sweep.txt
  GK_BNB_CAP=$1 GK_BNB_PRECAP=$2 GK_BNB_DEPTH=$3 timeout -k 10 120 python3 -u tools/bnb_time.py gap c5s_12x32 c5s_12x38 >> $O/sweep.txt 2>&1 || exit 1
done
