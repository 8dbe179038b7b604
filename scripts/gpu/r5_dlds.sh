#!/bin/bash
# Direct-to-LDS k-tiles for the NT bulk GEMM (PARSEC_GEMM_DLDS): numerics + kernel
# rate (unpadded and padded like the DPOTRF bulk streams), then configs 3 and 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/dlds; mkdir -p $O
for pad in 0 1; do for dl in 0 1; do
  PARSEC_GEMM_PAD_TEST=$pad PARSEC_GEMM_DLDS=$dl timeout -k 10 120 python3 scripts/kbench_gemm.py > $O/k_p${pad}_d${dl}.log 2>&1 || { echo "kbench pad=$pad dl=$dl failed"; tail -20 $O/k_p${pad}_d${dl}.log; exit 1; }
  echo "pad=$pad dl=$dl"; grep -E "gemm nb|gemm n=" $O/k_p${pad}_d${dl}.log
done; done
for dl in 0 1 0 1; do
  PARSEC_GEMM_DLDS=$dl timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > $O/c3_$dl.json 2> $O/c3_$dl.err || { tail -20 $O/c3_$dl.err; exit 1; }
  echo "c3 dl=$dl $(cut -c60-130 $O/c3_$dl.json) $(grep -o '"residual[^,]*' $O/c3_$dl.json)"
done
for dl in 0 1 0 1; do
  PARSEC_GEMM_DLDS=$dl timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > $O/c2_$dl.json 2> $O/c2_$dl.err || { tail -20 $O/c2_$dl.err; exit 1; }
  echo "c2 dl=$dl $(cut -c60-130 $O/c2_$dl.json) $(grep -o '"residual[^,]*' $O/c2_$dl.json)"
done
