#!/bin/bash
# DGEQRF 32k / nb 512: inner blocking ib 32 (default) vs 64 / 16, with the R check.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qib
for ib in 32 64 16 32; do
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --ib $ib --steps 2 --warmup 1 --check > gpurun_out/qib/ib$ib.json 2> gpurun_out/qib/ib$ib.err || { tail -5 gpurun_out/qib/ib$ib.err; exit 1; }
  echo "ib $ib $(cut -c60-110 gpurun_out/qib/ib$ib.json) $(grep -o '"residual[^,}]*' gpurun_out/qib/ib$ib.json)"
done
