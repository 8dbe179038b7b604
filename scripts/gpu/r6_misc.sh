#!/bin/bash
# Round 6: QR kernel profile, exact 8-rank pulled bytes, vectorised B-tile copies (tests + config 2/3).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/misc6; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
C2="--size 16384 --nb 512 --steps 5 --warmup 1"
AB_TAG=r6_vcopy bash scripts/gpu/bench_ab.sh "b;;$C2" "b2;;$C2" "b3;;$C2" "c3;;--steps 2 --warmup 1" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_multirank_gpu.py -k headline > $O/mr.log 2>&1 || { grep -E "assert|Error" $O/mr.log | head -5; tail -3 $O/mr.log; exit 1; }
tail -1 $O/mr.log
bash scripts/gpu/r6_qrprof.sh
