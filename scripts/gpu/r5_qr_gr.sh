#!/bin/bash
# DGEQRF 32k / nb 512: bulk group size (device_hip_group_rounds) A/B, alternating.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/qrg; mkdir -p $O
i=0
for g in 2 4 8 2 4 8 2 4; do
  i=$((i+1))
  PARSEC_MCA_device_hip_group_rounds=$g timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 > $O/q$i.json 2> $O/q$i.err || { echo "$g failed"; tail -5 $O/q$i.err; exit 1; }
  echo "group_rounds=$g $(grep -o '"value": [0-9.]*' $O/q$i.json)"
done
