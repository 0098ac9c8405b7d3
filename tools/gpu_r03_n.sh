#!/bin/bash
# C3 advance with the drift log (NS columns excluded), panel on and off
set -e
mkdir -p gpurun_out/r03n
GK_DRIFT_LOG=1 timeout -k 10 300 python3 -u tools/instab_probe.py 100000 > gpurun_out/r03n/drift_on.log 2>&1
GK_PANEL=0 GK_DRIFT_LOG=1 timeout -k 10 300 python3 -u tools/instab_probe.py 100000 > gpurun_out/r03n/drift_off.log 2>&1
echo ok
