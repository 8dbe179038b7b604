#!/bin/bash
# Staggered-start grouped GEMM (PARSEC_GEMM_STAGGER): kernel rates + error,
# GEMM kernel tests with it on, and DPOTRF A/B at configs 2 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stg
for st in 0 1; do
  for pad in 0 1; do
    echo "-- stagger $st pad $pad"
    PARSEC_GEMM_STAGGER=$st PARSEC_GEMM_PAD_TEST=$pad timeout -k 10 120 python3 scripts/kbench_gemm.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > gpurun_out/stg/rates.txt
cat gpurun_out/stg/rates.txt
PARSEC_GEMM_STAGGER=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py > gpurun_out/stg/tests.log 2>&1 || { tail -30 gpurun_out/stg/tests.log; exit 1; }
tail -2 gpurun_out/stg/tests.log
AB_TAG=r4_stagger bash scripts/gpu/bench_ab.sh \
 "s0_64;;--steps 2 --warmup 1" \
 "s1_64;PARSEC_GEMM_STAGGER=1;--steps 2 --warmup 1" \
 "s0_16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "s1_16;PARSEC_GEMM_STAGGER=1;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "s0b_64;;--steps 2 --warmup 1" \
 "s1b_64;PARSEC_GEMM_STAGGER=1;--steps 2 --warmup 1" || exit 1
