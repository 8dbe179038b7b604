#!/bin/bash
# Critical stream carrying ONLY the chain POTRF -> TRSM(k+1,k) -> SYRK(k,k+1)
# (hp_on_critical_stream 2: the other high-priority tasks get stream 1), with
# 1 or 2 bulk streams (2 bulk streams need a 5th hardware queue), +/- CU yield.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
H2="--mca device_hip_hp_on_critical_stream 2"
AB_TAG=r4_route bash scripts/gpu/bench_ab.sh \
 "b16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "h3_16;;--size 16384 --nb 512 --steps 5 --warmup 1 $H2 --mca device_hip_max_streams 3" \
 "h4_16;GPU_MAX_HW_QUEUES=8;--size 16384 --nb 512 --steps 5 --warmup 1 $H2 --mca device_hip_max_streams 4" \
 "h4y_16;GPU_MAX_HW_QUEUES=8;--size 16384 --nb 512 --steps 5 --warmup 1 $H2 --mca device_hip_max_streams 4 --mca device_hip_cu_yield 1" \
 "b4q8_16;GPU_MAX_HW_QUEUES=8;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "h3y_16;;--size 16384 --nb 512 --steps 5 --warmup 1 $H2 --mca device_hip_max_streams 3 --mca device_hip_cu_yield 1" \
 "b64;;--steps 2 --warmup 1" \
 "h4_64;GPU_MAX_HW_QUEUES=8;--steps 2 --warmup 1 $H2 --mca device_hip_max_streams 4" \
 "h3_64;;--steps 2 --warmup 1 $H2 --mca device_hip_max_streams 3" || exit 1
T16=t16h4 EXTRA="$H2 --mca device_hip_max_streams 4" GPU_MAX_HW_QUEUES=8 bash scripts/gpu/trace16.sh
