#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -k "qr" -p no:cacheprovider --timeout 60 --timeout-method thread > gpurun_out/qr_kernels.log 2>&1
rc1=$?
grep -E "PASSED|FAILED|ERROR|Timeout|passed|failed|Error|assert" gpurun_out/qr_kernels.log | tail -n 30 | cut -c1-250
if [ $rc1 -ne 124 ] && [ $rc1 -ne 137 ] && [ $rc1 -ne 139 ] && [ $rc1 -ne 134 ]; then
  PARSEC_MCA_debug_verbose=20 timeout -k 10 60 python -u scripts/qr_small.py > gpurun_out/qr_small.log 2>&1
  echo "== qr_small rc=$?"; grep -v "amdgpu.ids" gpurun_out/qr_small.log | tail -n 40 | cut -c1-200
fi
exit $rc1
