#!/bin/bash
# Blocked QR panels: kernel + taskpool numerics, then QR benches (progress to files).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
W="python benchmarks/bench_workloads.py"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dgeqrf.py -m gpu -x -v -k "qr or dgeqrf" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_qr.log 2>&1 && \
timeout -k 10 120 $W qr --n 4096 --nb 512 --steps 2 > gpurun_out/wl_qr4k.log 2>&1 && \
timeout -k 10 200 $W qr --n 8192 --nb 512 --steps 2 > gpurun_out/wl_qr8k.log 2>&1 && \
timeout -k 10 200 $W qr --n 16384 --nb 512 --steps 1 > gpurun_out/wl_qr16k.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|error" gpurun_out/pytest_qr.log | head -20 | cut -c1-200
for f in gpurun_out/wl_qr*.log; do echo "== $f"; grep "^{" $f | cut -c1-220; done
exit $rc
