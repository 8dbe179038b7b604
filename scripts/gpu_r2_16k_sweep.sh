#!/bin/bash
# DPOTRF 16k / nb 512 (BASELINE config 2): GEMM kernel-choice threshold sweep.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for bt in 384 192 96 32; do
  PARSEC_GEMM_BIG_TILES=$bt timeout -k 10 120 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/sw16_bt$bt.log 2>&1 || exit $?
  echo "bt=$bt $(grep -h '^{' gpurun_out/sw16_bt$bt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
