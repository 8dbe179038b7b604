#!/bin/bash
# 4 ranks sharing the box's one GPU: is the 32k slowdown GPU time-slicing of
# many process queues (theory) or the protocol? Same run with 2 HW queues per process.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PARSEC_BENCH_VERBOSE=1
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
timeout -k 10 150 $R --master-port 29571 bench.py --gpus 4 --size 16384 --nb 1024 --steps 2 --warmup 1 --share-gpu > gpurun_out/s4_16k.log 2>&1; echo "rc16=$?"; grep -h '^{' gpurun_out/s4_16k.log | cut -c1-200
GPU_MAX_HW_QUEUES=2 timeout -k 10 200 $R --master-port 29572 bench.py --gpus 4 --size 32768 --nb 1024 --steps 2 --warmup 1 --share-gpu > gpurun_out/s4_32k_q2.log 2>&1; echo "rc32q2=$?"; grep -h '^{' gpurun_out/s4_32k_q2.log | cut -c1-200
exit 0
