#!/bin/bash
# Vectorised stencil kernel + device-side initial condition: numerics tests,
# workload rate (1024^3, blocks 256 / 512) and a kernel trace.
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
W="python benchmarks/bench_workloads.py stencil"
timeout -k 10 300 python -u -m pytest tests/test_stencil3d.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/stencil_tests.log 2>&1 && \
timeout -k 10 300 $W --n 1024 --b 256 --iters 20 > gpurun_out/wl_stencil1024_b256.log 2>&1 && \
PARSEC_STENCIL_VEC=0 timeout -k 10 300 $W --n 1024 --b 256 --iters 20 > gpurun_out/wl_stencil1024_b256_scalar.log 2>&1 && \
timeout -k 10 300 $W --n 1024 --b 512 --iters 20 > gpurun_out/wl_stencil1024_b512.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/st1024v -o run -- python3 benchmarks/bench_workloads.py stencil --n 1024 --b 256 --iters 20 > gpurun_out/prof/st1024v.log 2>&1
rc=$?
tail -n 8 gpurun_out/stencil_tests.log
grep -h "^{" gpurun_out/wl_stencil*.log gpurun_out/prof/st1024v.log | cut -c1-300
exit $rc
