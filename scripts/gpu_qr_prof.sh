#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/qr8k -o run -- python3 benchmarks/bench_workloads.py qr --n 8192 --nb 512 --steps 1 > gpurun_out/prof/qr8k.log 2>&1 && \
timeout -k 10 300 python benchmarks/bench_workloads.py stencil --n 512 --b 128 --iters 20 > gpurun_out/wl_stencil512.log 2>&1 && \
timeout -k 10 300 python benchmarks/bench_workloads.py dtd_gemm --n 2048 --steps 2 > gpurun_out/wl_dtdgemm.log 2>&1
rc=$?
grep "^{" gpurun_out/prof/qr8k.log gpurun_out/wl_stencil512.log gpurun_out/wl_dtdgemm.log | cut -c1-250
exit $rc
