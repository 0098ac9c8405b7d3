#!/bin/bash
# MFMA panel pricing: forced-panel parity on the dense fixtures, C3 mid-solve
# windows with and without the panel, then the dense full solves (panel on by
# default from m = 1024)
set -e
mkdir -p gpurun_out/r03h
timeout -k 10 300 python -u -m pytest tests/test_panel.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r03h/panel_tests.log 2>&1
timeout -k 10 400 python3 -u tools/prof_panel.py 100000 10 32 > gpurun_out/r03h/panel_c3.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_lp.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or c3" > gpurun_out/r03h/lp_tests.log 2>&1
echo ok
