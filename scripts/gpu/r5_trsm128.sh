#!/bin/bash
# Panel-solve modes at nb 128 / 256 (host-published estimate route below 256).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/trsm128; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_dpotrf_gpu.py -m gpu -x -v -k "trsm_inverse_modes" --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -60 $O/test.log | cut -c1-300; exit 1; }
grep -E "PASSED|FAILED" $O/test.log | cut -c1-160; tail -1 $O/test.log
