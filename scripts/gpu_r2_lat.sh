#!/bin/bash
# multi-rank GPU tests + shared-GPU rank runs after the comm-thread polling change
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/mr_tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed" gpurun_out/mr_tests.log | tail -1
R2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 120 $R2 --master-port 29601 bench.py --gpus 2 --size 16384 --nb 1024 --steps 3 --warmup 1 --share-gpu --cores 2 > gpurun_out/s2_16k.log 2>&1; echo "rc=$?"; grep -h '^{' gpurun_out/s2_16k.log | cut -c1-200
R4="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
timeout -k 10 120 $R4 --master-port 29602 bench.py --gpus 4 --size 4096 --nb 1024 --steps 2 --warmup 1 --share-gpu --cores 2 > gpurun_out/s4_4k.log 2>&1; echo "rc=$?"; grep -h '^{' gpurun_out/s4_4k.log | cut -c1-200
exit 0
