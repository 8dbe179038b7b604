#!/bin/bash
# Per-panel critical chain of configs 2 and 3 from rocprofv3 kernel traces
set -o pipefail
mkdir -p gpurun_out/ch
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ch/t16 -o run -- python3 bench.py --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/ch/t16.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ch/t64 -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/ch/t64.log 2>&1
rc=$?
f=$(find gpurun_out/ch/t16 -name "*kernel_trace.csv" -print -quit); python3 scripts/critical_chain.py $f 512 16384 > gpurun_out/ch/chain16.txt; python3 scripts/trace_summary.py $f > gpurun_out/ch/sum16.txt
f=$(find gpurun_out/ch/t64 -name "*kernel_trace.csv" -print -quit); python3 scripts/critical_chain.py $f 1024 65536 > gpurun_out/ch/chain64.txt; python3 scripts/trace_summary.py $f > gpurun_out/ch/sum64.txt
rm -f $(find gpurun_out/ch -name "*kernel_trace.csv")
head -3 gpurun_out/ch/chain16.txt; tail -1 gpurun_out/ch/chain16.txt; head -3 gpurun_out/ch/chain64.txt; tail -1 gpurun_out/ch/chain64.txt; tail -1 gpurun_out/ch/sum16.txt; tail -1 gpurun_out/ch/sum64.txt
exit $rc
