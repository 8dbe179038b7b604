#!/bin/bash
# Round 5: grouped DGEMM "late C" epilogue (PARSEC_GEMM_LATE_C=1: C read into its
# own registers behind the first A/B tile, added at the end; one workgroup per CU
# launches only), kernel rates, then DPOTRF A/B at configs 2 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/latec; mkdir -p $O; : > $O/rate.txt
for l in 0 1; do for e in 0 -1; do
  echo "-- late_c $l epi $e pad 1" >> $O/rate.txt
  PARSEC_GEMM_LATE_C=$l PARSEC_GEMM_EPI=$e PARSEC_GEMM_PAD_TEST=1 timeout -k 10 120 python3 scripts/kbench_gemm.py >> $O/rate.txt 2>&1 || { tail -5 $O/rate.txt; exit 1; }
done; done
cat $O/rate.txt
AB_TAG=r5_latec bash scripts/gpu/bench_ab.sh \
 "base_16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "late_16;PARSEC_GEMM_LATE_C=1;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "base_16b;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "late_16b;PARSEC_GEMM_LATE_C=1;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "base_64;;--steps 2 --warmup 1" \
 "late_64;PARSEC_GEMM_EPI=2;--steps 2 --warmup 1" || exit 1
