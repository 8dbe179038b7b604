#!/bin/bash
# Round 6: in-place W-GEMM panel solve (no B copies, W read from the packed tile): tests, then A/B against the copy route.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/inpl; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py tests/test_trsm_modes.py > $O/t.log 2>&1 || { grep -E "FAILED|Error|error" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_inplace bash scripts/gpu/bench_ab.sh "ip;;$C2" "cp;PARSEC_TRSM_INPLACE=0;$C2" "ip2;;$C2" "cp2;PARSEC_TRSM_INPLACE=0;$C2" "ip3;;$C2" "cp3;PARSEC_TRSM_INPLACE=0;$C2" \
  "c3ip;;--steps 2 --warmup 1" "c3cp;PARSEC_TRSM_INPLACE=0;--steps 2 --warmup 1" || exit 1
