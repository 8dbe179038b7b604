#!/bin/bash
# One bulk GEMM workgroup per CU (device_hip_bulk_gemm_per_cu=1, padded LDS) vs
# two, with the 78 KB step kernel: kernel tests, critical latencies, configs 2, 3
set -o pipefail
mkdir -p gpurun_out/pc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/pc/ab.txt; : > $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py > gpurun_out/pc/kt.log 2>&1 || { tail -5 gpurun_out/pc/kt.log; exit 1; }
tail -1 gpurun_out/pc/kt.log
PARSEC_POTRF_STAMPS=1 timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/pc/kcrit.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/pc/kcrit.log
run() { local n=$1; shift
  timeout -k 10 240 python3 bench.py "$@" > gpurun_out/pc/$n.log 2>&1 || return 1
  echo "$n $* $(grep -h '^{' gpurun_out/pc/$n.log | cut -c90-150)" >> $out; }
run 16_c1 --size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_bulk_gemm_per_cu 1 &&
run 16_c2 --size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_bulk_gemm_per_cu 2 &&
run 16_c1b --size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_bulk_gemm_per_cu 1 &&
run 64_c2 --steps 2 --warmup 1 --mca device_hip_bulk_gemm_per_cu 2 &&
run 64_c1 --steps 2 --warmup 1 --mca device_hip_bulk_gemm_per_cu 1
rc=$?; cat $out; exit $rc
