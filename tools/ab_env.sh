#!/bin/bash
# A/B of bench.py's timed region under environment variants (experiments):
#   tools/ab_env.sh "VAR=1 VAR2=0" "VAR=2" ...   -> gpurun_out/ab_<i>.json
# every run has its own time limit; the script stops at the first failure
set -e
mkdir -p gpurun_out
i=0
for v in "$@"; do
  env $v timeout -k 10 300 python3 bench.py --no-cpu --no-extra > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$i.json').read().strip().splitlines()[-1])
print('$v'.ljust(40), d['value'], d['ms_per_step'], d['engine']['ms_split_per_step'])"
  i=$((i+1))
done
