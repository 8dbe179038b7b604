#!/bin/bash
# Two ranks on the box's one GPU (IPC plane between processes): throughput of
# the distributed path at scale, and 1-rank reference at the same size.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python bench.py --gpus 1 --size 32768 --nb 1024 --steps 2 --warmup 1 > gpurun_out/s1_32k.log 2>&1 && grep -h '^{' gpurun_out/s1_32k.log | cut -c1-260 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 \
    bench.py --gpus 2 --size 32768 --nb 1024 --steps 2 --warmup 1 --share-gpu > gpurun_out/s2_32k.log 2>&1 && grep -h '^{' gpurun_out/s2_32k.log | cut -c1-260 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29562 \
    bench.py --gpus 4 --size 32768 --nb 1024 --steps 2 --warmup 1 --share-gpu > gpurun_out/s4_32k.log 2>&1 && grep -h '^{' gpurun_out/s4_32k.log | cut -c1-260
