#!/bin/bash
# GPU programs (nvlink, DTD GPU chores) including the two-logical-device runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/logical; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_programs.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { grep -E "PASSED|FAILED|ERROR" $O/test.log | tail -20; tail -80 $O/test.log | cut -c1-300; exit 1; }
grep -E "PASSED|FAILED" $O/test.log | cut -c1-160; tail -2 $O/test.log
