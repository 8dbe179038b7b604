#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
timeout -k 10 180 python bench.py --size 8192 --nb 512 --steps 2 --warmup 1 --check --cores 4 > gpurun_out/c1_$i.log 2>&1 || { tail -5 gpurun_out/c1_$i.log; exit 1; }
echo "1 rank 8k/512: $(grep -o '"max_rel_error_vs_torch_cholesky": [0-9.e+-]*' gpurun_out/c1_$i.log)"
done
timeout -k 10 180 python bench.py --size 16384 --nb 512 --steps 2 --warmup 1 --check --cores 4 > gpurun_out/c1_16k.log 2>&1 || { tail -5 gpurun_out/c1_16k.log; exit 1; }
echo "1 rank 16k/512: $(grep -o '"max_rel_error_vs_torch_cholesky": [0-9.e+-]*' gpurun_out/c1_16k.log)"
timeout -k 10 180 python bench.py --size 8192 --nb 512 --steps 2 --warmup 1 --check --cores 1 > gpurun_out/c1_c1.log 2>&1 || { tail -5 gpurun_out/c1_c1.log; exit 1; }
echo "1 rank 8k/512 cores 1: $(grep -o '"max_rel_error_vs_torch_cholesky": [0-9.e+-]*' gpurun_out/c1_c1.log)"
