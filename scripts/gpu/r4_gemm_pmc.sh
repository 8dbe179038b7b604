#!/bin/bash
# Grouped DGEMM 40 x 1024^3: throughput (kbench_gemm) and PMC passes on the
# shipped 128x128 kernel, unpadded (2 workgroups / CU) and padded as the DPOTRF
# bulk streams launch it (1 workgroup / CU: PARSEC_GEMM_PAD_TEST=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gpmc
: > gpurun_out/gpmc/rate.txt
for v in 0 9 10; do
  for pad in 0 1; do
    echo "-- variant $v pad $pad" >> gpurun_out/gpmc/rate.txt
    PARSEC_GEMM_VARIANT=$v PARSEC_GEMM_PAD_TEST=$pad timeout -k 10 120 python3 scripts/kbench_gemm.py >> gpurun_out/gpmc/rate.txt 2>&1 || { tail -5 gpurun_out/gpmc/rate.txt; exit 1; }
  done
done
: > gpurun_out/gpmc/rate_pad.txt
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
P2="FETCH_SIZE TCC_HIT_sum SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for tag in nopad pad; do
  if [ $tag = pad ]; then export PARSEC_GEMM_PAD_TEST=1; else unset PARSEC_GEMM_PAD_TEST; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/gpmc/${tag}_p$i -o run -- python3 scripts/kbench_gemm_only.py > gpurun_out/gpmc/${tag}_p$i.log 2>&1 || { echo "pmc $tag pass $i failed"; tail -5 gpurun_out/gpmc/${tag}_p$i.log; exit 1; }
  done
done
unset PARSEC_GEMM_PAD_TEST
for f in $(find gpurun_out/gpmc -name "*counter_collection.csv"); do python3 scripts/pmc_summary.py $f dgemm_batch_kernel; done > gpurun_out/gpmc/summary.txt
cat gpurun_out/gpmc/rate.txt gpurun_out/gpmc/rate_pad.txt gpurun_out/gpmc/summary.txt
AB_TAG=r4_gemm_variants bash scripts/gpu/bench_ab.sh \
 "v0_64;;--steps 2 --warmup 1" \
 "v9_64;PARSEC_GEMM_VARIANT=9;--steps 2 --warmup 1" \
 "v10_64;PARSEC_GEMM_VARIANT=10;--steps 2 --warmup 1" \
 "v0_16;;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "v9_16;PARSEC_GEMM_VARIANT=9;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "v10_16;PARSEC_GEMM_VARIANT=10;--size 16384 --nb 512 --steps 5 --warmup 1" \
 "inv64;PARSEC_DPOTRF_TRSM=inverse;--steps 2 --warmup 1" || exit 1
