#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for x in 0 3 7; do
PARSEC_MCA_device_hip_critical_streams=$x timeout -k 10 300 python benchmarks/bench_workloads.py qr --n 16384 --nb 512 --steps 2 > gpurun_out/ab_qr_$x.log 2>&1 || exit 1
echo "qr16k xcrit=$x $(grep -o '"value": [0-9.]*' gpurun_out/ab_qr_$x.log)"
done
for x in 0 3; do
for r in 1 2; do
PARSEC_MCA_device_hip_critical_streams=$x timeout -k 10 240 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_64k_$x.log 2>&1 || exit 1
echo "potrf64k xcrit=$x $(grep -o '"value": [0-9.]*' gpurun_out/ab_64k_$x.log)"
PARSEC_MCA_device_hip_critical_streams=$x timeout -k 10 240 python bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/ab_16k_$x.log 2>&1 || exit 1
echo "potrf16k xcrit=$x $(grep -o '"value": [0-9.]*' gpurun_out/ab_16k_$x.log)"
done
done
