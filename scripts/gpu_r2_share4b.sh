#!/bin/bash
# 4 ranks sharing the one GPU with 1 worker thread each (CPU threads <= the box's 16-CPU share)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PARSEC_BENCH_VERBOSE=1
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
timeout -k 10 150 $R --master-port 29581 bench.py --gpus 4 --size 16384 --nb 1024 --steps 2 --warmup 1 --share-gpu --cores 1 > gpurun_out/s4_16k_c1.log 2>&1; echo "rc=$?"; grep -h '^{' gpurun_out/s4_16k_c1.log | cut -c1-200
timeout -k 10 170 $R --master-port 29582 bench.py --gpus 4 --size 32768 --nb 1024 --steps 1 --warmup 1 --share-gpu --cores 1 > gpurun_out/s4_32k_c1.log 2>&1; echo "rc=$?"; grep -h '^{' gpurun_out/s4_32k_c1.log | cut -c1-200
exit 0
