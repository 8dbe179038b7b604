#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof/qrt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof/qrt -o run -- python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 1 > gpurun_out/prof/qrt.log 2>&1
rc=$?
f=$(find gpurun_out/prof/qrt -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_summary.py $f
exit $rc
