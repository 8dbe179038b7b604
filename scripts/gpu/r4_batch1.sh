#!/bin/bash
# One box for: grouped-GEMM variants + PMC, DGEQRF wave-priority A/B, 4-rank stencil.
set -o pipefail
bash scripts/gpu/r4_gemm_pmc.sh > gpurun_out/batch1_gemm.log 2>&1 || { tail -20 gpurun_out/batch1_gemm.log; exit 1; }
tail -30 gpurun_out/batch1_gemm.log
bash scripts/gpu/r4_qr.sh || exit 1
bash scripts/gpu/r4_stencil4.sh || exit 1
