#!/bin/bash
# Critical chain at config 2 with the cooperative CU yield on (1: POTRF steps
# claim; 2: every critical-group kernel claims).
set -o pipefail
T16=t16y1 EXTRA="--mca device_hip_cu_yield 1" bash scripts/gpu/trace16.sh || exit 1
T16=t16y2 EXTRA="--mca device_hip_cu_yield 2" bash scripts/gpu/trace16.sh || exit 1
