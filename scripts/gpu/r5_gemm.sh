#!/bin/bash
# Round 5: grouped DGEMM with the atomic epilogue (PARSEC_GEMM_EPI=1: C += alpha AB
# through memory-side f64 adds, no C preload) and the persistent grid
# (PARSEC_GEMM_PERSIST=1), kernel rates then DPOTRF A/B at configs 3 and 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gemm; mkdir -p $O; : > $O/rate.txt
for e in 0 1; do for p in 0 1; do for pad in 1 0; do
  echo "-- epi $e persist $p pad $pad" >> $O/rate.txt
  PARSEC_GEMM_EPI=$e PARSEC_GEMM_PERSIST=$p PARSEC_GEMM_PAD_TEST=$pad timeout -k 10 120 python3 scripts/kbench_gemm.py >> $O/rate.txt 2>&1 || { tail -5 $O/rate.txt; exit 1; }
done; done; done
cat $O/rate.txt
AB_TAG=r5_gemm_epi bash scripts/gpu/bench_ab.sh \
 "e0p0_64;;--steps 2 --warmup 1" \
 "e1p0_64;PARSEC_GEMM_EPI=1;--steps 2 --warmup 1" \
 "e1p1_64;PARSEC_GEMM_EPI=1 PARSEC_GEMM_PERSIST=1;--steps 2 --warmup 1" \
 "e0p1_64;PARSEC_GEMM_PERSIST=1;--steps 2 --warmup 1" \
 "e0p0_16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "e1p0_16;PARSEC_GEMM_EPI=1;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "e1p1_16;PARSEC_GEMM_EPI=1 PARSEC_GEMM_PERSIST=1;--size 16384 --nb 512 --steps 5 --warmup 1" || exit 1
