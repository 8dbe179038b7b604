#!/bin/bash
# DGEQRF 32k / nb 512: bulk groups in flight (1 = round-4 default, 2) and bulk GEMM
# workgroups per CU (1 padded = default, 2) A/B, plus the --check residual once.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qrk
for spec in "m1;" "m2;PARSEC_MCA_device_hip_max_inflight_batches=2" "p2;PARSEC_MCA_device_hip_bulk_gemm_per_cu=2" "m3;PARSEC_MCA_device_hip_max_inflight_batches=3" \
            "m1b;" "m2b;PARSEC_MCA_device_hip_max_inflight_batches=2" "p2b;PARSEC_MCA_device_hip_bulk_gemm_per_cu=2" "m3b;PARSEC_MCA_device_hip_max_inflight_batches=3"; do
  IFS=';' read -r name envs <<< "$spec"
  env X_AB=1 $envs timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 > gpurun_out/qrk/$name.json 2> gpurun_out/qrk/$name.err || { tail -5 gpurun_out/qrk/$name.err; exit 1; }
  echo "$name [$envs] $(cut -c1-110 gpurun_out/qrk/$name.json)"
done
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 1 --warmup 1 --check > gpurun_out/qrk/check.json 2> gpurun_out/qrk/check.err || { tail -5 gpurun_out/qrk/check.err; exit 1; }
cut -c1-400 gpurun_out/qrk/check.json
