#!/bin/bash
# Multi-rank validation on a 1-GPU box: ranks share GPU 0, shm data plane.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PARSEC_BENCH_VERBOSE=1
PARSEC_MCA_debug_verbose=10 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --size 2048 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 3 > gpurun_out/multi2s.log 2>&1 && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
    bench.py --gpus 2 --size 8192 --nb 512 --steps 2 --warmup 1 --share-gpu --check --cores 3 > gpurun_out/multi2.log 2>&1 && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29535 \
    bench.py --gpus 4 --size 8192 --nb 512 --steps 2 --warmup 1 --share-gpu --check --cores 2 > gpurun_out/multi4.log 2>&1
rc=$?
for f in gpurun_out/multi2s.log gpurun_out/multi2.log gpurun_out/multi4.log; do echo "== $f"; grep -v "amdgpu.ids\|socket.cpp" $f | tail -n 30 | cut -c1-300; done
exit $rc
