#!/bin/bash
# Cooperative CU yield (device_hip_cu_yield): DPOTRF correctness with the yield
# on, then A/B at config 2 (16k / nb 512) and config 3 (64k / nb 1024).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
PARSEC_MCA_device_hip_cu_yield=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dpotrf_gpu.py > gpurun_out/ab/yield_tests.log 2>&1 || { tail -20 gpurun_out/ab/yield_tests.log; exit 1; }
tail -2 gpurun_out/ab/yield_tests.log
AB_TAG=r4_yield bash scripts/gpu/bench_ab.sh \
 "b16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "y1_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_cu_yield 1" \
 "y2_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_cu_yield 2" \
 "y2s_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_cu_yield 2 --mca device_hip_critical_split 1" \
 "b64;;--steps 2 --warmup 1" \
 "y1_64;;--steps 2 --warmup 1 --mca device_hip_cu_yield 1" \
 "y2_64;;--steps 2 --warmup 1 --mca device_hip_cu_yield 2" || exit 1
