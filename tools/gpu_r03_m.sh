#!/bin/bash
# panel tests (age variants); C3 advance with the drift and growth log
set -e
mkdir -p gpurun_out/r03m
timeout -k 10 300 python -u -m pytest tests/test_panel.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03m/panel_tests.log 2>&1
GK_DRIFT_LOG=1 timeout -k 10 300 python3 -u tools/instab_probe.py 100000 > gpurun_out/r03m/drift.log 2>&1
echo ok
