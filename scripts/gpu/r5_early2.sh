#!/bin/bash
# Round 5: early release variants (1 = critical-path tasks only, 2 = every
# critical-stream task) at config 2, manager timings (PARSEC_BENCH_VERBOSE).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PARSEC_BENCH_VERBOSE=1
AB_TAG=r5_early2 bash scripts/gpu/bench_ab.sh \
 "b16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "e1_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 1" \
 "e2_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 2" \
 "e1h2_16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 1 --mca device_hip_hp_on_critical_stream 2" \
 "b16r;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "e1_16r;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 1" || exit 1
for f in b16 e1_16 e2_16 e1h2_16; do echo "$f $(grep -o '"manager_ms.*' gpurun_out/ab/$f.log)"; done
