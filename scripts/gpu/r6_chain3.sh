#!/bin/bash
# Round 6: critical-release dispatch (critical successors launched before the rest of a retired group is released), alone and with routes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hops
PARSEC_MCA_device_hip_critical_release=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dpotrf_gpu.py -m gpu -k "hbm or trsm" > gpurun_out/hops/t_cr.log 2>&1 || { tail -20 gpurun_out/hops/t_cr.log; exit 1; }
tail -1 gpurun_out/hops/t_cr.log
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
CR="--mca device_hip_critical_release 1"
AB_TAG=r6_chain3 bash scripts/gpu/bench_ab.sh "b;;$C2" "cr;;$C2 $CR" "crs;;$C2 $CR --mca device_hip_critical_split 1" \
  "crh2;GPU_MAX_HW_QUEUES=8;$C2 $CR --mca device_hip_hp_on_critical_stream 2 --mca device_hip_max_streams 4" \
  "b2;;$C2" "cr2;;$C2 $CR" "crla3;PARSEC_DPOTRF_SYRK_LOOKAHEAD=3;$C2 $CR" "b3;;$C2" "cr3;;$C2 $CR" "c3;;--steps 2 --warmup 1" "c3cr;;--steps 2 --warmup 1 $CR" || exit 1
