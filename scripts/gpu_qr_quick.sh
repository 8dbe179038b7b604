#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgeqrf.py -m gpu -k "qr" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_qr.log 2>&1
rc=$?; tail -n 1 gpurun_out/pytest_qr.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_qr.log | head -20; exit $rc; }
timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 2 > gpurun_out/wl_qr16k.log 2>&1 && grep '^{' gpurun_out/wl_qr16k.log | cut -c1-150 && \
timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 1 > gpurun_out/wl_qr32k.log 2>&1 && grep '^{' gpurun_out/wl_qr32k.log | cut -c1-150
