#!/bin/bash
# DGEQRF config 4 (32k / nb 512): per-kernel time of one factorization.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qrt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qrt/prof -o run -- python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 1 --warmup 1 > gpurun_out/qrt/prof.log 2>&1 || { tail -5 gpurun_out/qrt/prof.log; exit 1; }
f=$(find gpurun_out/qrt/prof -name "*kernel_stats.csv" -print -quit)
cp $f gpurun_out/qrt/kernel_stats.csv
t=$(find gpurun_out/qrt/prof -name "*kernel_trace.csv" -print -quit)
python3 scripts/trace_summary.py $t > gpurun_out/qrt/summary.txt 2>&1 || true
rm -rf gpurun_out/qrt/prof
head -12 gpurun_out/qrt/kernel_stats.csv | cut -c1-200; cat gpurun_out/qrt/summary.txt | head -20
