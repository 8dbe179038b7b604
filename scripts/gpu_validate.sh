#!/bin/bash
# Round validation: GPU tests, smoke, 2-rank shared-GPU bench (device IPC data plane), 1-GPU benches, kernel profile.
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --size 4096 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 3 > gpurun_out/multi2s.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/bench_16k.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench_64k.log 2>&1
rc=$?
for f in gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/multi2s.log gpurun_out/bench_*.log; do echo "== $f"; tail -n 6 $f | grep -v amdgpu.ids | cut -c1-400; done
exit $rc
