#!/bin/bash
# Round 6: host hops on the config-2 chain, then A/B: SYRK(k-1,k) fused into POTRF(k), critical-first dispatch, 64x64 critical tiles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu/r6_hops.sh || exit 1
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dpotrf_gpu.py -m gpu > gpurun_out/hops/t.log 2>&1 || { tail -20 gpurun_out/hops/t.log; exit 1; }
tail -1 gpurun_out/hops/t.log
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_chain2 bash scripts/gpu/bench_ab.sh "b;;$C2" "fs;PARSEC_DPOTRF_FUSE_SYRK=1;$C2" "cf;;$C2 --mca device_hip_critical_first 1" "ct;PARSEC_CRIT_TILE=64;$C2" \
  "b2;;$C2" "fs2;PARSEC_DPOTRF_FUSE_SYRK=1;$C2" "fscf;PARSEC_DPOTRF_FUSE_SYRK=1;$C2 --mca device_hip_critical_first 1" "fsct;PARSEC_DPOTRF_FUSE_SYRK=1 PARSEC_CRIT_TILE=64;$C2" \
  "b3;;$C2" "fs3;PARSEC_DPOTRF_FUSE_SYRK=1;$C2" "c3;;--steps 2 --warmup 1" "c3fs;PARSEC_DPOTRF_FUSE_SYRK=1;--steps 2 --warmup 1" || exit 1
