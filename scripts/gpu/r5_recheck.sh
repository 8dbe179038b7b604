#!/bin/bash
# Headline re-check at the final state: 4 bench runs on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/recheck; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py > $O/c3_$i.json 2> $O/c3_$i.err || { tail -5 $O/c3_$i.err; exit 1; }
  echo "c3 run $i $(grep -o '"value": [0-9.]*' $O/c3_$i.json)"
done
rocm-smi --showclocks 2>/dev/null | grep -iE "sclk|mclk" | head -4 || true
