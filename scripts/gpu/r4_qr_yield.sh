#!/bin/bash
# DGEQRF config 4 with the cooperative CU yield: the TS chain's sub-panel kernels
# claim their CUs, bulk GEMM workgroups there pause (device_hip_cu_yield).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qry
PARSEC_MCA_device_hip_cu_yield=1 timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 8192 --nb 512 --steps 1 --warmup 0 --check > gpurun_out/qry/check.json 2> gpurun_out/qry/check.err || { tail -5 gpurun_out/qry/check.err; exit 1; }
cut -c1-400 gpurun_out/qry/check.json
for spec in "y0;PARSEC_MCA_device_hip_cu_yield=0" "y1;PARSEC_MCA_device_hip_cu_yield=1" "y0b;PARSEC_MCA_device_hip_cu_yield=0" "y1b;PARSEC_MCA_device_hip_cu_yield=1"; do
  IFS=';' read -r name envs <<< "$spec"
  env $envs timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 > gpurun_out/qry/$name.json 2> gpurun_out/qry/$name.err || { tail -5 gpurun_out/qry/$name.err; exit 1; }
  echo "$name $envs $(cut -c1-120 gpurun_out/qry/$name.json)"
done
