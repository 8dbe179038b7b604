#!/bin/bash
# 4-rank stencil + 2-rank QR cold runs after the blocking-stream device_memcpy fix.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/sq_mr.log 2>&1; rc=$?
tail -n 2 gpurun_out/sq_mr.log
[ $rc -ne 0 ] && exit $rc
RUNS=16 bash scripts/gpu_r2_qrcold.sh
