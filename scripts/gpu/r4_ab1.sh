#!/bin/bash
# Round-4 first GPU pass: critical-path engine knobs and evenly spread CU
# reservations at configs 2 and 3, then the multi-rank tests of the CE path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AB_TAG=r4_ab1 bash scripts/gpu/bench_ab.sh \
 "b16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "s16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_critical_split 1" \
 "sc16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_critical_split 1 --mca device_hip_critical_bulk_cap 1" \
 "r8_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_reserved_cus 8" \
 "r16_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_reserved_cus 16" \
 "r16x_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_reserved_cus 16 --mca device_hip_reserved_cus_exclusive 1" \
 "b64;;--steps 2 --warmup 1" \
 "s64;;--steps 2 --warmup 1 --mca device_hip_critical_split 1" \
 "r8_64;;--steps 2 --warmup 1 --mca device_hip_reserved_cus 8" || exit 1
bash scripts/gpu/multirank.sh
