#!/bin/bash
# DTD stencil: wall-clock rate at 1024^3 (block 256) and a kernel trace of the
# same run, to split kernel time from runtime gaps.
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
W="python benchmarks/bench_workloads.py stencil"
timeout -k 10 300 $W --n 1024 --b 256 --iters 20 > gpurun_out/wl_stencil1024_b256.log 2>&1 && \
timeout -k 10 300 $W --n 1024 --b 512 --iters 20 > gpurun_out/wl_stencil1024_b512.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/st1024 -o run -- python3 benchmarks/bench_workloads.py stencil --n 1024 --b 256 --iters 20 > gpurun_out/prof/st1024.log 2>&1
rc=$?
grep -h "^{" gpurun_out/wl_stencil*.log gpurun_out/prof/st1024.log | cut -c1-300
exit $rc
