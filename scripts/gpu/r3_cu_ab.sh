#!/bin/bash
# CU partition A/B: critical stream on R reserved CUs (stride S), bulk on the rest
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3/cu_ab.txt; : > $out
for cfg in "0 1" "16 1" "16 8" "16 32" "32 8" "8 32"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 --mca device_hip_reserved_cus $1 --mca device_hip_reserved_cus_stride $2 > gpurun_out/r3/cu_$1_$2.log 2>&1 || exit 1
  echo "16k R=$1 stride=$2 $(grep -h '^{' gpurun_out/r3/cu_$1_$2.log | cut -c90-140)" >> $out
done
cat $out
