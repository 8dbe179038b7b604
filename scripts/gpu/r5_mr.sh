#!/bin/bash
# Multi-rank GPU tests + GPU memory tests after the unpin change.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/mr; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_multirank_gpu.py tests/test_gpu_memory.py tests/test_gpu_programs.py -m gpu -x -v --timeout 250 --timeout-method thread > $O/test.log 2>&1 || { grep -E "PASSED|FAILED|ERROR" $O/test.log | tail -20; tail -50 $O/test.log | cut -c1-300; exit 1; }
grep -cE "PASSED" $O/test.log; tail -1 $O/test.log
