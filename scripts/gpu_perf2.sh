#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/bench_16k.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 3 --warmup 1 --mca device_hip_reserved_cus 0 > gpurun_out/bench_16k_nomask.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench_64k.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/p16k -o run -- python3 bench.py --gpus 1 --n 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/prof/bench16k.log 2>&1
rc=$?
for f in gpurun_out/pytest_gpu.log gpurun_out/kbench.log gpurun_out/bench_*.log; do echo "== $f"; tail -n 20 $f | grep -v amdgpu.ids | cut -c1-300; done
exit $rc
