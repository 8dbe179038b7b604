#!/bin/bash
# Three-buffer direct-to-LDS bulk GEMM (PARSEC_GEMM_VARIANT=12 + PARSEC_GEMM_DLDS=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/dlds3; mkdir -p $O
for spec in "0 0" "0 1" "12 1" "0 0" "12 1"; do
  set -- $spec
  PARSEC_GEMM_VARIANT=$1 PARSEC_GEMM_PAD_TEST=1 PARSEC_GEMM_DLDS=$2 timeout -k 10 120 python3 scripts/kbench_gemm.py > $O/k_v$1_d$2.log 2>&1 || { echo "kbench $spec failed"; tail -20 $O/k_v$1_d$2.log; exit 1; }
  echo "v=$1 dl=$2"; grep -E "gemm nb|gemm n=" $O/k_v$1_d$2.log
done
for spec in "0 0" "12 1" "0 0" "12 1"; do
  set -- $spec
  PARSEC_GEMM_VARIANT=$1 PARSEC_GEMM_DLDS=$2 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > $O/c3_$1_$2.json 2> $O/c3_$1_$2.err || { tail -20 $O/c3_$1_$2.err; exit 1; }
  echo "c3 v=$1 dl=$2 $(cut -c60-130 $O/c3_$1_$2.json) $(grep -o '"residual[^,]*' $O/c3_$1_$2.json)"
done
