#!/bin/bash
# Multi-rank GPU tests (all ranks share the box's GPU) + the CE C program.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py -m gpu -v -x -p no:cacheprovider --timeout 280 --timeout-method thread > gpurun_out/multirank.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Timeout|passed|failed|rank .* dpotrf" gpurun_out/multirank.log | tail -n 30 | cut -c1-250
exit $rc
