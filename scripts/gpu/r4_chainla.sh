#!/bin/bash
# Config 2 (16k / nb 512): the chain's lookahead inputs (SYRK(k, k+2), GEMM(k+2, k+1, k))
# at the critical threshold (PARSEC_DPOTRF_SYRK_LOOKAHEAD=2), with the three routes of the
# other high-priority work (critical stream / least-loaded bulk stream / own stream).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r4_chainla bash scripts/gpu/bench_ab.sh \
 "base;;$B" "la1;PARSEC_DPOTRF_SYRK_LOOKAHEAD=1;$B" "la2;PARSEC_DPOTRF_SYRK_LOOKAHEAD=2;$B" \
 "hp0;;$B --mca device_hip_hp_on_critical_stream 0" "hp0la2;PARSEC_DPOTRF_SYRK_LOOKAHEAD=2;$B --mca device_hip_hp_on_critical_stream 0" \
 "hp2la2;PARSEC_DPOTRF_SYRK_LOOKAHEAD=2 GPU_MAX_HW_QUEUES=8;$B --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4" \
 "cspla2;PARSEC_DPOTRF_SYRK_LOOKAHEAD=2;$B --mca device_hip_critical_split 1" \
 "base_b;;$B" "la2_b;PARSEC_DPOTRF_SYRK_LOOKAHEAD=2;$B" "hp0la2_b;PARSEC_DPOTRF_SYRK_LOOKAHEAD=2;$B --mca device_hip_hp_on_critical_stream 0" \
 "hp2la2_b;PARSEC_DPOTRF_SYRK_LOOKAHEAD=2 GPU_MAX_HW_QUEUES=8;$B --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4" || exit 1
