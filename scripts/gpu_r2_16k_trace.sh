#!/bin/bash
# Kernel timeline of DPOTRF 16k / nb 512 (config 2): GPU busy fraction and concurrency
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/p16 -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/prof/p16.log 2>&1
rc=$?; grep -h '^{' gpurun_out/prof/p16.log | cut -c1-200; exit $rc
