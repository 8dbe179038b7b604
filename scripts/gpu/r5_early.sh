#!/bin/bash
# Round 5: early release of critical-stream groups (device_hip_early_release):
# correctness tests, then DPOTRF A/B at configs 2 and 3 with hp routes 1 / 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/early; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_dpotrf_gpu.py -x -v --timeout 200 --timeout-method thread -k "early or hbm or trsm_inverse" > $O/test.log 2>&1 || { grep -E "PASSED|FAILED|Error|error" $O/test.log | tail -20; tail -40 $O/test.log | cut -c1-300; exit 1; }
grep -cE "PASSED" $O/test.log; tail -1 $O/test.log
AB_TAG=r5_early bash scripts/gpu/bench_ab.sh \
 "b16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "e16;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 1" \
 "e16h2;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 1 --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_inflight_batches 2" \
 "e16cs;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 1 --mca device_hip_critical_split 1" \
 "b64;;--steps 2 --warmup 1" \
 "e64;;--steps 2 --warmup 1 --mca device_hip_early_release 1" \
 "b16r;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "e16r;;--size 16384 --nb 512 --steps 5 --warmup 1 --mca device_hip_early_release 1" || exit 1
