#!/bin/bash
# the multi-rank bench path (2 ranks sharing the GPU: gloo + the TCP comm)
set -e
mkdir -p gpurun_out/r03o
GK_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r03o/bench2.json 2> gpurun_out/r03o/bench2.err
echo ok
