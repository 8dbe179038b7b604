#!/bin/bash
# QR chain kernels held at <= 128 VGPRs (fit beside a bulk GEMM workgroup):
# numerics, config-4 rate, kernel trace; then max_inflight_batches 1 vs 2 at 16k/64k.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qrcap
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "qr or geqrf" --timeout 200 --timeout-method thread > gpurun_out/qrcap/tests.log 2>&1 || { tail -30 gpurun_out/qrcap/tests.log; exit 1; }
tail -1 gpurun_out/qrcap/tests.log
for name in a b; do
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 > gpurun_out/qrcap/$name.json 2> gpurun_out/qrcap/$name.err || { tail -5 gpurun_out/qrcap/$name.err; exit 1; }
  echo "qr32 $name $(cut -c1-160 gpurun_out/qrcap/$name.json)"
done
bash scripts/gpu/r4_qr_trace.sh || exit 1
B="--size 16384 --nb 512 --steps 5 --warmup 1"
C="--steps 3 --warmup 1"
AB_TAG=r4_inflight bash scripts/gpu/bench_ab.sh \
 "m2_16;;$B" "m1_16;;$B --mca device_hip_max_inflight_batches 1" \
 "m2_16b;;$B" "m1_16b;;$B --mca device_hip_max_inflight_batches 1" \
 "m2_64;;$C" "m1_64;;$C --mca device_hip_max_inflight_batches 1" || exit 1
