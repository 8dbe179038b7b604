#!/bin/bash
# TRSM inverse/auto/blocked modes on the GPU, the 4-rank stencil halo path, and
# a bench A/B of the panel-solve modes at configs 2 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trsm
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dpotrf_gpu.py "tests/test_multirank_gpu.py::test_stencil_four_ranks_ipc" > gpurun_out/trsm/tests.log 2>&1 || { tail -30 gpurun_out/trsm/tests.log; exit 1; }
tail -3 gpurun_out/trsm/tests.log
AB_TAG=r4_trsm_modes bash scripts/gpu/bench_ab.sh \
 "auto16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "inv16;PARSEC_DPOTRF_TRSM=inverse;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "blk16;PARSEC_DPOTRF_TRSM=blocked;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "auto64;;--steps 2 --warmup 1" \
 "inv64;PARSEC_DPOTRF_TRSM=inverse;--steps 2 --warmup 1" \
 "blk64;PARSEC_DPOTRF_TRSM=blocked;--steps 2 --warmup 1" || exit 1
