#!/bin/bash
# A/B: GPU task release on compute threads (device_hip_complete_on_workers) and
# the pending-task storage, 16k/nb512 and 64k/nb1024, interleaved; then the GPU suite.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab2.log
run() {  # tag size nb steps warmup env...
  local tag=$1 n=$2 nb=$3 st=$4 wu=$5; shift 5
  timeout -k 10 300 env "$@" python bench.py --gpus 1 --size $n --nb $nb --steps $st --warmup $wu > gpurun_out/ab2_$tag.log 2>&1 || return $?
  echo "$tag $(grep -h '"metric"' gpurun_out/ab2_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/ab2.log
}
for rep in 1 2; do
  run cow16_$rep 16384 512 6 2 PARSEC_MCA_device_hip_complete_on_workers=1 || exit $?
  run mgr16_$rep 16384 512 6 2 PARSEC_MCA_device_hip_complete_on_workers=0 || exit $?
  run cowhash16_$rep 16384 512 6 2 PARSEC_MCA_device_hip_complete_on_workers=1 PARSEC_MCA_ptg_dep_management=dynamic-hash-table || exit $?
done
run cow64 65536 1024 3 1 PARSEC_MCA_device_hip_complete_on_workers=1 || exit $?
run mgr64 65536 1024 3 1 PARSEC_MCA_device_hip_complete_on_workers=0 || exit $?
cat gpurun_out/ab2.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/ab2_tests.log
exit $rc
