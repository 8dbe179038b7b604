#!/bin/bash
# CU reservation A/B at config 2: R CUs (stride S) kept free of bulk work;
# exclusive = critical stream on those only, shared = critical stream on all CUs
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3/cu_ab.txt; : > $out
for cfg in "0 1 0" "8 32 0" "16 16 0" "32 8 0" "16 16 1" "8 32 1" "0 1 0"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 4 --warmup 1 --mca device_hip_reserved_cus $1 --mca device_hip_reserved_cus_stride $2 --mca device_hip_reserved_cus_exclusive $3 > gpurun_out/r3/cu_$1_$2_$3.log 2>&1 || exit 1
  echo "16k R=$1 stride=$2 excl=$3 $(grep -h '^{' gpurun_out/r3/cu_$1_$2_$3.log | cut -c90-150)" >> $out
done
for cfg in "0 1 0" "8 32 0"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --mca device_hip_reserved_cus $1 --mca device_hip_reserved_cus_stride $2 --mca device_hip_reserved_cus_exclusive $3 > gpurun_out/r3/cu64_$1_$2_$3.log 2>&1 || exit 1
  echo "64k R=$1 stride=$2 excl=$3 $(grep -h '^{' gpurun_out/r3/cu64_$1_$2_$3.log | cut -c90-150)" >> $out
done
cat $out
