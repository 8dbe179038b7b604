#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/q
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 scripts/qr_sub2_phases.py > gpurun_out/q/ph.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/q/ph.log; exit $rc
