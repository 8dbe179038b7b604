#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for nb in 256 384; do
timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 16384 --nb $nb --steps 1 > gpurun_out/wl_qr16k_nb$nb.log 2>&1 || exit $?
grep '^{' gpurun_out/wl_qr16k_nb$nb.log | cut -c1-200
done
