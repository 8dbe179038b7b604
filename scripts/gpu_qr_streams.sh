#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_dgeqrf.py tests/test_dpotrf_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_qr.log 2>&1 && tail -n 1 gpurun_out/pytest_qr.log && \
timeout -k 10 200 python benchmarks/bench_workloads.py qr --n 8192 --nb 512 --steps 2 > gpurun_out/wl_qr8k.log 2>&1 && grep '^{' gpurun_out/wl_qr8k.log | cut -c1-150 && \
timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 2 > gpurun_out/wl_qr16k.log 2>&1 && grep '^{' gpurun_out/wl_qr16k.log | cut -c1-150 && \
timeout -k 10 200 python bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/bench_16k.log 2>&1 && grep '^{' gpurun_out/bench_16k.log | cut -c1-150 && \
timeout -k 10 240 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_64k.log 2>&1 && grep '^{' gpurun_out/bench_64k.log | cut -c1-150
