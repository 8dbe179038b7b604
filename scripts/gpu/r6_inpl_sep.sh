#!/bin/bash
# Round 6: in-place W-GEMM in its own kernel instantiation (bulk NT code as before): tests, configs 3 / 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/isep; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dpotrf_gpu.py tests/test_kernels_gpu.py tests/test_headline_gpu.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
AB_TAG=r6_isep bash scripts/gpu/bench_ab.sh "c3;;--steps 3 --warmup 1" "c3b;;--steps 3 --warmup 1" "c2;;--size 16384 --nb 512 --steps 5 --warmup 1" "c2b;;--size 16384 --nb 512 --steps 5 --warmup 1" "c3c;;--steps 3 --warmup 1" || exit 1
