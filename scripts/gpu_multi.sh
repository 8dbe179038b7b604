#!/bin/bash
# GPU tests, then multi-rank validation on a 1-GPU box (ranks share GPU 0, shm data plane).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 PARSEC_BENCH_VERBOSE=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
PARSEC_MCA_debug_verbose=10 timeout -k 10 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --size 2048 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 3 > gpurun_out/multi2s.log 2>&1
rc=$?
echo "== pytest"; tail -n 30 gpurun_out/pytest_gpu.log | cut -c1-300
echo "== multi2s"; grep -v "amdgpu.ids\|socket.cpp\|comm\]" gpurun_out/multi2s.log | tail -n 20 | cut -c1-300
exit $rc
