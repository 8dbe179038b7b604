#!/bin/bash
# Kernel trace of the critical-path micro-benchmark (per-dispatch durations)
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/kp -o run -- python3 scripts/kbench_critical.py > gpurun_out/r3/kp.log 2>&1
rc=$?; cat gpurun_out/r3/kp.log | tail -6; exit $rc
