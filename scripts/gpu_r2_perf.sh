#!/bin/bash
# DPOTRF 16k/nb512: GEMM big-tile threshold sweep
set -o pipefail
export PYTHONUNBUFFERED=1
for bt in 384 192 96 0; do
  echo "== big_tiles $bt"
  PARSEC_GEMM_BIG_TILES=$bt timeout -k 10 200 python bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 2>&1 | grep -v amdgpu | cut -c1-200
done
echo "== big_tiles 0, 6 exec streams"
PARSEC_GEMM_BIG_TILES=0 timeout -k 10 200 python bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 --mca device_hip_max_streams 6 2>&1 | grep -v amdgpu | cut -c1-200
