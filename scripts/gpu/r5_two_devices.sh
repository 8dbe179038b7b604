#!/bin/bash
# DPOTRF over two logical devices of one GPU + the GPU programs' two-device tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/two; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_memory.py tests/test_gpu_programs.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { grep -E "two_devices|PASSED|FAILED" $O/test.log | tail -20; tail -40 $O/test.log | cut -c1-300; exit 1; }
grep -E "two_devices N=|PASSED|FAILED" $O/test.log | cut -c1-300; tail -1 $O/test.log
