#!/bin/bash
# BASELINE configs 1, 4, 5 on one MI355X (QR, DTD stencil, DTD DGEMM on CPU) + QR kernel profile.
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
W="python benchmarks/bench_workloads.py"
timeout -k 10 300 $W qr --n 8192 --nb 512 --steps 2 > gpurun_out/wl_qr8k.log 2>&1 && \
timeout -k 10 300 $W qr --n 16384 --nb 512 --steps 2 > gpurun_out/wl_qr16k.log 2>&1 && \
timeout -k 10 300 $W stencil --n 512 --b 128 --iters 20 > gpurun_out/wl_stencil512.log 2>&1 && \
timeout -k 10 300 $W dtd_gemm --n 2048 --steps 2 > gpurun_out/wl_dtdgemm.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/qr16k -o run -- python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 1 > gpurun_out/prof/qr16k.log 2>&1
rc=$?
for f in gpurun_out/wl_*.log gpurun_out/prof/qr16k.log; do echo "== $f"; grep "^{" $f | cut -c1-260; tail -n 2 $f | grep -v "^{" | cut -c1-200; done
exit $rc
