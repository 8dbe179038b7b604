#!/bin/bash
# Cooperative CU yield (device_hip_cu_yield 1 / 2) on top of the one-bulk-group default, config 2 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--size 16384 --nb 512 --steps 5 --warmup 1"
C="--steps 3 --warmup 1"
AB_TAG=r4_yield_m1 bash scripts/gpu/bench_ab.sh \
 "b16;;$B" "y1_16;;$B --mca device_hip_cu_yield 1" "y2_16;;$B --mca device_hip_cu_yield 2" \
 "b16b;;$B" "y1_16b;;$B --mca device_hip_cu_yield 1" "y2_16b;;$B --mca device_hip_cu_yield 2" \
 "b64;;$C" "y1_64;;$C --mca device_hip_cu_yield 1" || exit 1
