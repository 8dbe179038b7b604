#!/bin/bash
# DGEQRF 32k / nb 512: hierarchical (default) vs the flat-TS taskpool (ib 32 / 64).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qfl
for spec in "hqr;--qr-tree hqr" "flat32;--qr-tree flat --ib 32" "flat64;--qr-tree flat --ib 64" "hqr2;--qr-tree hqr" "flat32b;--qr-tree flat --ib 32"; do
  IFS=';' read -r name a <<< "$spec"
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 --check $a > gpurun_out/qfl/$name.json 2> gpurun_out/qfl/$name.err || { tail -5 gpurun_out/qfl/$name.err; exit 1; }
  echo "$name $(cut -c60-110 gpurun_out/qfl/$name.json) $(grep -o '"residual[^,}]*' gpurun_out/qfl/$name.json)"
done
