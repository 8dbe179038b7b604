#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgeqrf.py -m gpu -k "qr" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_qr.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_qr.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_qr.log | head -20; exit $rc; }
PARSEC_QR_PANEL_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "qr" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_qr4.log 2>&1
rc=$?; tail -n 1 gpurun_out/pytest_qr4.log; [ $rc -eq 0 ] || exit $rc
PARSEC_QR_PROFILE=1 timeout -k 5 100 python scripts/qr_tsqrt_only.py && \
timeout -k 10 120 python scripts/qr_kbench.py 512 && \
PARSEC_QR_PANEL_WAVES=4 timeout -k 10 120 python scripts/qr_kbench.py 512 && \
timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 2 > gpurun_out/wl_qr16k.log 2>&1 && grep '^{' gpurun_out/wl_qr16k.log | cut -c1-150
