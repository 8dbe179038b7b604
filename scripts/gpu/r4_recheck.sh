#!/bin/bash
# Re-measure config 2 and QR 32k (a validation run read 39.6 / 24.9 TF).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rc
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > gpurun_out/rc/b16_$i.json 2> gpurun_out/rc/b16_$i.err || { tail -20 gpurun_out/rc/b16_$i.err; exit 1; }
  echo "b16 $i $(cut -c80-140 gpurun_out/rc/b16_$i.json)"
done
for i in 1 2; do
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 2 --warmup 1 > gpurun_out/rc/qr_$i.json 2> gpurun_out/rc/qr_$i.err || { tail -5 gpurun_out/rc/qr_$i.err; exit 1; }
  echo "qr $i $(cut -c60-120 gpurun_out/rc/qr_$i.json)"
done
rocm-smi --showclocks --showpower 2>/dev/null | head -20 || true
