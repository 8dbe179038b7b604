#!/bin/bash
# Stencil output stores: non-temporal vs plain, 1024^3 blocks 256; numerics tests first
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
W="python benchmarks/bench_workloads.py stencil --n 1024 --b 256 --iters 20"
timeout -k 10 200 python -u -m pytest tests/test_stencil3d.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/st_tests.log 2>&1 && tail -n 2 gpurun_out/st_tests.log && \
for nt in 1 0 1 0; do PARSEC_STENCIL_NT=$nt timeout -k 10 200 $W > gpurun_out/st_nt$nt.log 2>&1 || exit $?; echo "nt=$nt $(grep -h '^{' gpurun_out/st_nt$nt.log | cut -c1-120)"; done
