#!/bin/bash
# DGEQRF 32k / nb 512 engine knobs not swept before (group_rounds, sort_pending, max_streams, hp route).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/qrk; mkdir -p $O
i=0
for e in "X=0" "PARSEC_MCA_device_hip_group_rounds=1" "PARSEC_MCA_device_hip_group_rounds=4" "PARSEC_MCA_device_hip_sort_pending_tasks=2" "PARSEC_MCA_device_hip_max_streams=4" "PARSEC_MCA_device_hip_hp_on_critical_stream=0" "X=0"; do
  i=$((i+1))
  env $e timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 > $O/q$i.json 2> $O/q$i.err || { echo "$e failed"; tail -5 $O/q$i.err; exit 1; }
  echo "$e $(grep -o '"value": [0-9.]*' $O/q$i.json)"
done
