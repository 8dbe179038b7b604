#!/bin/bash
# Vendor batched DGEMM for uniform bulk tile batches: tests, then A/B at
# configs 3 and 2 (PARSEC_GEMM_VENDOR, device_hip_vendor_gemm_min_dim)
set -o pipefail
mkdir -p gpurun_out/g
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/g/vendor_ab.txt; : > $out
PARSEC_GEMM_VENDOR=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py > gpurun_out/g/kt.log 2>&1 || { tail -5 gpurun_out/g/kt.log; exit 1; }
tail -1 gpurun_out/g/kt.log
run() { local n=$1 e=$2; shift 2
  env $e timeout -k 10 240 python3 bench.py "$@" > gpurun_out/g/$n.log 2>&1 || return 1
  echo "$n $e $* $(grep -h '^{' gpurun_out/g/$n.log | cut -c90-150)" >> $out; }
run 64_v1 PARSEC_GEMM_VENDOR=1 --steps 3 --warmup 1 &&
run 64_v0 PARSEC_GEMM_VENDOR=0 --steps 3 --warmup 1 &&
run 64_v1b PARSEC_GEMM_VENDOR=1 --steps 3 --warmup 1 &&
run 16_v0 PARSEC_GEMM_VENDOR=0 --size 16384 --nb 512 --steps 5 --warmup 1 &&
run 16_v512 PARSEC_GEMM_VENDOR=1 --size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_vendor_gemm_min_dim 512 &&
timeout -k 10 120 python3 scripts/kbench_gemm_vs_vendor.py > gpurun_out/g/kvv.log 2>&1
rc=$?; cat $out; grep -v amdgpu gpurun_out/g/kvv.log | tail -6; exit $rc
