#!/bin/bash
# Round validation: GPU tests, smoke, 8-rank shared-GPU rehearsal of the
# P4xQ2 grid over the IPC plane, then the default bench and config 2.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/gpu_tests.sh && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -n 2 gpurun_out/smoke.log && \
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 \
    bench.py --gpus 8 --size 8192 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 1 > gpurun_out/multi8s.log 2>&1 && \
grep '^{' gpurun_out/multi8s.log && \
timeout -k 10 240 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/bench_64k.log 2>&1 && grep '^{' gpurun_out/bench_64k.log && \
timeout -k 10 120 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/bench_16k.log 2>&1 && grep '^{' gpurun_out/bench_16k.log
