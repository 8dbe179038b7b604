#!/bin/bash
# Run-to-run spread of the headline (config 3) and config 2 on one box: 8 bench runs each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/stats; mkdir -p $O
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 300 python3 bench.py > $O/c3_$i.json 2> $O/c3_$i.err || { tail -5 $O/c3_$i.err; exit 1; }
  echo "c3 run $i $(grep -o '"value": [0-9.]*' $O/c3_$i.json) $(grep -o '"ms_per_step": [0-9.]*' $O/c3_$i.json)"
done
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 2 > $O/c2_$i.json 2> $O/c2_$i.err || { tail -5 $O/c2_$i.err; exit 1; }
  echo "c2 run $i $(grep -o '"value": [0-9.]*' $O/c2_$i.json) $(grep -o '"ms_per_step": [0-9.]*' $O/c2_$i.json)"
done
