#!/bin/bash
# Kernel trace of config 2 (DPOTRF 16k / nb 512, jdf taskpool) for the per-panel critical chain
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/t16 -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 --taskpool jdf > gpurun_out/r3/t16.log 2>&1
rc=$?; grep -h '^{' gpurun_out/r3/t16.log | cut -c1-200; exit $rc
