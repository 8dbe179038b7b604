#!/bin/bash
# GPU manager polls without sleeping while work is in flight: 16k and 64k DPOTRF
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/p16a.log 2>&1 && grep -h '^{' gpurun_out/p16a.log | cut -c1-200 && \
timeout -k 10 120 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/p16b.log 2>&1 && grep -h '^{' gpurun_out/p16b.log | cut -c1-200 && \
timeout -k 10 240 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/p64.log 2>&1 && grep -h '^{' gpurun_out/p64.log | cut -c1-200
