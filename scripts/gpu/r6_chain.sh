#!/bin/bash
# Round 6: config-2 critical-chain routes with the one-panel lookahead set
# critical (PARSEC_DPOTRF_SYRK_LOOKAHEAD=3) and the cost of the packed panel tile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_chain bash scripts/gpu/bench_ab.sh \
 "b;;$C2" \
 "np;PARSEC_POTRF_PACK=0;$C2" \
 "la3;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2" \
 "la3h0;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0" \
 "la3h2;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3 GPU_MAX_HW_QUEUES=8;$C2 --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4" \
 "la3h0r16x;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0 --mca device_hip_reserved_cus 16 --mca device_hip_reserved_cus_exclusive 1" \
 "la3h0r32x;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0 --mca device_hip_reserved_cus 32 --mca device_hip_reserved_cus_exclusive 1" \
 "la3h2r32x;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3 GPU_MAX_HW_QUEUES=8;$C2 --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4 --mca device_hip_reserved_cus 32 --mca device_hip_reserved_cus_exclusive 1" \
 "la3h0r32;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 --mca device_hip_hp_on_critical_stream 0 --mca device_hip_reserved_cus 32" \
 "b2;;$C2" \
 "np2;PARSEC_POTRF_PACK=0;$C2" || exit 1
