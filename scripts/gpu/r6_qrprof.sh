#!/bin/bash
# Round 6: DGEQRF config 4 kernel trace summary (timed factorization).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/qrp6; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 1 --warmup 1 > $O/q.log 2>&1 || { tail -5 $O/q.log; exit 1; }
t=$(find $O/t -name "*kernel_trace.csv" -print -quit)
python3 scripts/trace_summary.py $t > $O/summary.txt 2>&1; cat $O/summary.txt
gzip -c $t > $O/trace.csv.gz; rm -rf $O/t
