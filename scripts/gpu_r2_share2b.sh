#!/bin/bash
# 2 ranks on the one GPU after the comm-thread on/off change
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 150 $R2 --master-port 29631 bench.py --gpus 2 --size 16384 --nb 1024 --steps 3 --warmup 1 --share-gpu --cores 2 --check > gpurun_out/s2_16k_final.log 2>&1 && grep -h '^{' gpurun_out/s2_16k_final.log | cut -c1-220 && \
timeout -k 10 150 $R2 --master-port 29632 bench.py --gpus 2 --size 32768 --nb 1024 --steps 2 --warmup 1 --share-gpu > gpurun_out/s2_32k_final.log 2>&1 && grep -h '^{' gpurun_out/s2_32k_final.log | cut -c1-220
