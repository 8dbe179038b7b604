#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qrp
timeout -k 10 200 python3 scripts/qr_sub2_phases.py > gpurun_out/qrp/idle.txt 2>&1 || { tail -5 gpurun_out/qrp/idle.txt; exit 1; }
timeout -k 10 300 python3 scripts/qr_phases_loaded.py 32768 > gpurun_out/qrp/loaded.txt 2>&1 || { tail -5 gpurun_out/qrp/loaded.txt; exit 1; }
PARSEC_MCA_device_hip_cu_yield=1 timeout -k 10 300 python3 scripts/qr_phases_loaded.py 32768 > gpurun_out/qrp/loaded_yield.txt 2>&1 || { tail -5 gpurun_out/qrp/loaded_yield.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/qrp/idle.txt; grep -v amdgpu.ids gpurun_out/qrp/loaded.txt; grep -v amdgpu.ids gpurun_out/qrp/loaded_yield.txt
