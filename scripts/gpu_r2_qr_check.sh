#!/bin/bash
# DGEQRF (BASELINE config 4 shape) on 1 GPU with the R-factor check at benchmark scale.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 --check > gpurun_out/qr32k_check.log 2>&1 && grep -h '^{' gpurun_out/qr32k_check.log && \
timeout -k 10 200 python benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 3 --warmup 1 --check > gpurun_out/qr16k_check.log 2>&1 && grep -h '^{' gpurun_out/qr16k_check.log
