#!/bin/bash
# Tile-POTRF change check: kernel tests, critical-kernel latencies with phase
# stamps, configs 2 and 3
set -o pipefail
mkdir -p gpurun_out/k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py > gpurun_out/k/kt.log 2>&1 &&
PARSEC_POTRF_STAMPS=1 timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/k/kstamps.log 2>&1 &&
timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > gpurun_out/k/b16.log 2>&1 &&
timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 > gpurun_out/k/b64.log 2>&1
rc=$?; tail -2 gpurun_out/k/kt.log; grep -v amdgpu gpurun_out/k/kstamps.log; grep -h '^{' gpurun_out/k/b16.log gpurun_out/k/b64.log | cut -c1-200; exit $rc
