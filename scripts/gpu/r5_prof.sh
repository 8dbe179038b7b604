#!/bin/bash
# Round 5 closing profiles: MFMA-busy PMC of the grouped GEMM with the atomic
# epilogue (the config-3 default) against the preload epilogue, both padded as the
# DPOTRF bulk streams launch them; kernel statistics of configs 3 and 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/prof5; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
export PARSEC_GEMM_PAD_TEST=1
for e in 0 1; do
  PARSEC_GEMM_EPI=$e timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/epi$e -o run -- python3 scripts/kbench_gemm_only.py > $O/epi$e.log 2>&1 || { echo "pmc epi $e failed"; tail -5 $O/epi$e.log; exit 1; }
done
unset PARSEC_GEMM_PAD_TEST
for f in $(find $O -name "*counter_collection.csv"); do python3 scripts/pmc_summary.py $f dgemm_batch_kernel; done > $O/pmc_summary.txt
cat $O/pmc_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 bench.py --steps 1 --warmup 1 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
f=$(find $O/c3 -name "*kernel_stats.csv" -print -quit); cp $f $O/c3_kernel_stats.csv; rm -rf $O/c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
f=$(find $O/c2 -name "*kernel_stats.csv" -print -quit); cp $f $O/c2_kernel_stats.csv; rm -rf $O/c2
head -8 $O/c3_kernel_stats.csv | cut -c1-200; head -8 $O/c2_kernel_stats.csv | cut -c1-200
grep -h '^{' $O/c3.log $O/c2.log | cut -c1-200
