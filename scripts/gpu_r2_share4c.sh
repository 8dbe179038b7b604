#!/bin/bash
# 4 ranks on the one GPU, small N, comm debug log with timestamps
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PARSEC_BENCH_VERBOSE=1 PARSEC_MCA_debug_verbose=10
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
timeout -k 10 120 $R --master-port 29591 bench.py --gpus 4 --size 4096 --nb 1024 --steps 2 --warmup 1 --share-gpu --cores 2 > gpurun_out/s4_4k_dbg.log 2>&1; echo "rc=$?"; grep -h '^{' gpurun_out/s4_4k_dbg.log | cut -c1-200
export PARSEC_MCA_debug_verbose=0
R2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 120 $R2 --master-port 29592 bench.py --gpus 2 --size 16384 --nb 1024 --steps 2 --warmup 1 --share-gpu --cores 2 > gpurun_out/s2_16k.log 2>&1; echo "rc=$?"; grep -h '^{' gpurun_out/s2_16k.log | cut -c1-200
exit 0
