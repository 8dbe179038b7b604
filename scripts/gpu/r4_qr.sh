#!/bin/bash
# DGEQRF config 4 (32k / nb 512, 1 GPU): wave priority of the TS chain's
# sub-panel kernels (PARSEC_QR_PRIO) A/B, then a kernel trace of the winner.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qr
for spec in "p0;PARSEC_QR_PRIO=0" "p1;PARSEC_QR_PRIO=1" "p0b;PARSEC_QR_PRIO=0" "p1b;PARSEC_QR_PRIO=1"; do
  IFS=';' read -r name envs <<< "$spec"
  env $envs timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 > gpurun_out/qr/$name.json 2> gpurun_out/qr/$name.err || { tail -5 gpurun_out/qr/$name.err; exit 1; }
  echo "$name $envs $(cut -c1-120 gpurun_out/qr/$name.json)"
done
