#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgeqrf.py -m gpu -k "qr" -v -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_qr.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Error|assert|passed|failed" gpurun_out/pytest_qr.log | tail -n 30 | cut -c1-250
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/qr_kbench.py 512 > gpurun_out/qr_kbench.log 2>&1 && cat gpurun_out/qr_kbench.log && \
timeout -k 10 200 python benchmarks/bench_workloads.py qr --n 8192 --nb 512 --steps 2 > gpurun_out/wl_qr8k.log 2>&1 && grep '^{' gpurun_out/wl_qr8k.log && \
timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 2 > gpurun_out/wl_qr16k.log 2>&1 && grep '^{' gpurun_out/wl_qr16k.log
