#!/bin/bash
# DGEQRF 16k: kernel-trace summaries of the flat TS tree and the hierarchical
# tree (TS domains of 4 + TT binary trees)
set -o pipefail
mkdir -p gpurun_out/h
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in 0 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/h/d$d -o run -- python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 1 --qr-domain $d > gpurun_out/h/d$d.log 2>&1 || exit 1
  f=$(find gpurun_out/h/d$d -name "*kernel_trace.csv" -print -quit)
  python3 scripts/trace_summary.py $f > gpurun_out/h/sum_d$d.txt
  grep -h '^{' gpurun_out/h/d$d.log | cut -c1-160; cat gpurun_out/h/sum_d$d.txt
done
