#!/bin/bash
# DGEQRF taskpool bulk-inflight hint (2) vs an explicit device_hip_max_inflight_batches=1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qrh
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "qr or geqrf" --timeout 200 --timeout-method thread > gpurun_out/qrh/tests.log 2>&1 || { tail -30 gpurun_out/qrh/tests.log; exit 1; }
tail -1 gpurun_out/qrh/tests.log
for spec in "w;" "h;" "x1;PARSEC_MCA_device_hip_max_inflight_batches=1" "h2;" "x1b;PARSEC_MCA_device_hip_max_inflight_batches=1" "h3;"; do
  IFS=';' read -r name envs <<< "$spec"
  env X_AB=1 $envs timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 > gpurun_out/qrh/$name.json 2> gpurun_out/qrh/$name.err || { tail -5 gpurun_out/qrh/$name.err; exit 1; }
  echo "$name [$envs] $(cut -c1-110 gpurun_out/qrh/$name.json)"
done
