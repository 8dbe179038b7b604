#!/bin/bash
# BK=32 bulk GEMM (PARSEC_GEMM_VARIANT=11) with / without direct-to-LDS k-tiles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/dlds2; mkdir -p $O
for v in 0 11; do for dl in 0 1; do
  PARSEC_GEMM_VARIANT=$v PARSEC_GEMM_PAD_TEST=1 PARSEC_GEMM_DLDS=$dl timeout -k 10 120 python3 scripts/kbench_gemm.py > $O/k_v${v}_d${dl}.log 2>&1 || { echo "kbench v=$v dl=$dl failed"; tail -20 $O/k_v${v}_d${dl}.log; exit 1; }
  echo "v=$v dl=$dl"; grep -E "gemm nb|gemm n=" $O/k_v${v}_d${dl}.log
done; done
for spec in "0 0" "11 1" "0 1" "11 1" "11 0"; do
  set -- $spec
  PARSEC_GEMM_VARIANT=$1 PARSEC_GEMM_DLDS=$2 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > $O/c3_$1_$2.json 2> $O/c3_$1_$2.err || { tail -20 $O/c3_$1_$2.err; exit 1; }
  echo "c3 v=$1 dl=$2 $(cut -c60-130 $O/c3_$1_$2.json) $(grep -o '"residual[^,]*' $O/c3_$1_$2.json)"
done
for spec in "0 0" "11 1" "0 0" "11 1"; do
  set -- $spec
  PARSEC_GEMM_VARIANT=$1 PARSEC_GEMM_DLDS=$2 timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > $O/c2_$1_$2.json 2> $O/c2_$1_$2.err || { tail -20 $O/c2_$1_$2.err; exit 1; }
  echo "c2 v=$1 dl=$2 $(cut -c60-130 $O/c2_$1_$2.json) $(grep -o '"residual[^,]*' $O/c2_$1_$2.json)"
done
