#!/bin/bash
# Instability probe on C3 (tools/instab_probe.py): panel age cap default (100),
# no cap, panel off
set -e
mkdir -p gpurun_out/r03j
timeout -k 10 200 python3 -u tools/instab_probe.py 64000 > gpurun_out/r03j/age100.log 2>&1
GK_PANEL_AGE=100000000 timeout -k 10 200 python3 -u tools/instab_probe.py 64000 > gpurun_out/r03j/nocap.log 2>&1
GK_PANEL=0 timeout -k 10 200 python3 -u tools/instab_probe.py 64000 > gpurun_out/r03j/off.log 2>&1
echo ok
