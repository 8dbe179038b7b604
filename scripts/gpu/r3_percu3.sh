#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pc3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PARSEC_GEMM_PAD_DEBUG=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pc3/t -o run -- python3 bench.py --size 16384 --nb 512 --steps 2 --warmup 1 --mca device_hip_bulk_gemm_per_cu 1 > gpurun_out/pc3/t.log 2>&1 || exit 1
f=$(find gpurun_out/pc3/t -name "*kernel_trace.csv" -print -quit)
python3 scripts/critical_chain.py $f 512 16384 > gpurun_out/pc3/chain.txt; head -12 gpurun_out/pc3/chain.txt; tail -1 gpurun_out/pc3/chain.txt
python3 scripts/trace_summary.py $f | head -4
rm -f $f
grep -h "\[gemm\]" gpurun_out/pc3/t.log | head -2
