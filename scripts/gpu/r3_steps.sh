#!/bin/bash
# Step-fused tile POTRF: numerics, phase clocks, config 2 (+ kernel trace) and config 3
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/r3/kt.log 2>&1 &&
PARSEC_POTRF_STAMPS=1 timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/r3/kstamps.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/t16 -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/r3/t16.log 2>&1 &&
timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/r3/b16.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/r3/b64.log 2>&1
rc=$?; tail -2 gpurun_out/r3/kt.log; grep "^n=" gpurun_out/r3/kstamps.log; for f in gpurun_out/r3/t16.log gpurun_out/r3/b16.log gpurun_out/r3/b64.log; do echo $f; grep -h '^{' $f | cut -c1-200; done; exit $rc
