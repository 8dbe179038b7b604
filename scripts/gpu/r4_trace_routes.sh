#!/bin/bash
# Launch logs + kernel traces at config 2: default engine (one bulk group in flight)
# and the pure-chain route with the lookahead inputs critical.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T16=t16m1 bash scripts/gpu/trace16.sh || exit 1
export PARSEC_DPOTRF_SYRK_LOOKAHEAD=2 GPU_MAX_HW_QUEUES=8
T16=t16h2la EXTRA="--mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4" bash scripts/gpu/trace16.sh || exit 1
