#!/bin/bash
# End-to-end A/B of the direct-to-LDS bulk GEMM (PARSEC_GEMM_DLDS) at configs 3 and 2, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/dlds4; mkdir -p $O
i=0
for dl in 0 1 0 1 0 1; do
  i=$((i+1))
  PARSEC_GEMM_DLDS=$dl timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > $O/c3_$i.json 2> $O/c3_$i.err || { tail -20 $O/c3_$i.err; exit 1; }
  echo "c3 dl=$dl $(grep -o '"value": [0-9.]*' $O/c3_$i.json)"
done
for dl in 0 1 0 1 0 1; do
  i=$((i+1))
  PARSEC_GEMM_DLDS=$dl timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > $O/c2_$i.json 2> $O/c2_$i.err || { tail -20 $O/c2_$i.err; exit 1; }
  echo "c2 dl=$dl $(grep -o '"value": [0-9.]*' $O/c2_$i.json)"
done
