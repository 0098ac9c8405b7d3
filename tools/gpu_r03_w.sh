#!/bin/bash
# round profile of the final pivot kernels (tools/profile_round.sh r03)
set -e
timeout -k 10 1500 bash tools/profile_round.sh r03 > gpurun_out/profile_round_r03.log 2>&1
echo ok
