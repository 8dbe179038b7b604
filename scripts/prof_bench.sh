#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/p16k -o run -- python3 bench.py --gpus 1 --n 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/prof/bench16k.log 2>&1
rc=$?
find gpurun_out/prof -name "*stats*" | head
exit $rc
