#!/bin/bash
# PMC counters of the grouped 128x128 DGEMM kernel (one rocprofv3 pass per counter group).
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/t -o run -- python3 scripts/kbench_gemm_only.py > gpurun_out/pmc/t.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 scripts/kbench_gemm_only.py > gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc/p2 -o run -- python3 scripts/kbench_gemm_only.py > gpurun_out/pmc/p2.log 2>&1
rc=$?
ls -R gpurun_out/pmc | head -30
exit $rc
