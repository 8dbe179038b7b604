#!/bin/bash
# Round 6: copy route restored as default; the in-place W-GEMM as an opt-in (tests both, A/B).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/inpl; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py tests/test_trsm_modes.py > $O/t_def.log 2>&1 || { grep -E "FAILED|Error" $O/t_def.log | head; tail -5 $O/t_def.log; exit 1; }
tail -1 $O/t_def.log
PARSEC_TRSM_INPLACE=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dpotrf_gpu.py tests/test_trsm_modes.py > $O/t_ip.log 2>&1 || { grep -E "FAILED|Error" $O/t_ip.log | head; tail -5 $O/t_ip.log; exit 1; }
tail -1 $O/t_ip.log
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_inplace2 bash scripts/gpu/bench_ab.sh "b;;$C2" "ip;PARSEC_TRSM_INPLACE=1;$C2" "b2;;$C2" "b3;;$C2" "c3;;--steps 2 --warmup 1" "c3ip;PARSEC_TRSM_INPLACE=1;--steps 2 --warmup 1" "c3b;;--steps 2 --warmup 1" || exit 1
