#!/bin/bash
# Config 3 (64k / nb 1024): rocprofv3 kernel trace -> per-panel critical chain.
set -o pipefail
mkdir -p gpurun_out/t64
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/t64/prof -o run -- python3 bench.py --steps 1 --warmup 1 $EXTRA > gpurun_out/t64/prof.log 2>&1 || { tail -5 gpurun_out/t64/prof.log; exit 1; }
f=$(find gpurun_out/t64/prof -name "*kernel_trace.csv" -print -quit)
python3 scripts/critical_chain.py $f 1024 65536 > gpurun_out/t64/chain64.txt
rm -rf gpurun_out/t64/prof
head -3 gpurun_out/t64/chain64.txt; tail -1 gpurun_out/t64/chain64.txt; grep -h '^{' gpurun_out/t64/prof.log | cut -c1-200
