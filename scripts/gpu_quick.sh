#!/bin/bash
# Quick GPU validation: GPU tests, kernel micro-benchmarks, 16k and 64k bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/kbench.py > gpurun_out/kbench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/bench_16k.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/bench_16k_b.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench_64k.log 2>&1
rc=$?
for f in gpurun_out/pytest_gpu.log gpurun_out/kbench.log gpurun_out/bench_*.log; do echo "== $f"; tail -n 20 $f | grep -v amdgpu.ids | cut -c1-250; done
exit $rc
