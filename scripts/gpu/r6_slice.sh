#!/bin/bash
# Round 6: bulk groups retired in slices (device_hip_retire_slice) so critical completions are noticed between slices.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/slice; mkdir -p $O
PARSEC_MCA_device_hip_retire_slice=8 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dpotrf_gpu.py tests/test_gpu_memory.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_slice bash scripts/gpu/bench_ab.sh "b;;$C2" "s8;;$C2 --mca device_hip_retire_slice 8" "s32;;$C2 --mca device_hip_retire_slice 32" \
  "b2;;$C2" "s8b;;$C2 --mca device_hip_retire_slice 8" "s32b;;$C2 --mca device_hip_retire_slice 32" "b3;;$C2" "s8c;;$C2 --mca device_hip_retire_slice 8" \
  "c3;;--steps 2 --warmup 1" "c3s8;;--steps 2 --warmup 1 --mca device_hip_retire_slice 8" || exit 1
