#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "potrf or trsm_through" > gpurun_out/r3/kt.log 2>&1 &&
PARSEC_POTRF_STAMPS=1 timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/r3/kstamps.log 2>&1
rc=$?; tail -2 gpurun_out/r3/kt.log; cat gpurun_out/r3/kstamps.log; exit $rc
