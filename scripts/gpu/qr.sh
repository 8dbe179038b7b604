#!/bin/bash
# Column-owner QR sub-panel kernel: QR kernel / DGEQRF GPU tests, isolated
# TSQRT latency, DGEQRF 16k / 32k (vs PARSEC_QR_SUB2=0)
set -o pipefail
mkdir -p gpurun_out/c
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dgeqrf.py -k "qr or geqrf" > gpurun_out/c/t.log 2>&1
rc0=$?; tail -2 gpurun_out/c/t.log; grep -E "FAILED|Error" gpurun_out/c/t.log | head -5
[ $rc0 -eq 0 ] &&
timeout -k 10 120 python3 scripts/qr_kbench.py 512 > gpurun_out/c/k1.log 2>&1 &&
PARSEC_QR_SUB2=0 timeout -k 10 120 python3 scripts/qr_kbench.py 512 > gpurun_out/c/k0.log 2>&1 &&
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 2 --check > gpurun_out/c/q16.log 2>&1 &&
PARSEC_QR_SUB2=0 timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 2 > gpurun_out/c/q16_0.log 2>&1 &&
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 1 --check > gpurun_out/c/q32.log 2>&1
rc=$?; grep -h "TSQRT\|GEQRT" gpurun_out/c/k1.log gpurun_out/c/k0.log; grep -h '^{' gpurun_out/c/q*.log | cut -c1-300; exit $((rc0+rc))
