#!/bin/bash
# Routing / manager A/B at config 2: high-priority tasks on the critical stream or the
# bulk streams, completion release on the manager or on the workers, bulk depth
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3/route_ab.txt; : > $out
export PARSEC_BENCH_VERBOSE=1
i=0
for cfg in "hp_on_critical_stream 0" "hp_on_critical_stream 1" "complete_on_workers 1" "max_inflight_batches 4" "max_inflight_batches 1"; do
  set -- $cfg; i=$((i+1))
  timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 --mca device_hip_$1 $2 > gpurun_out/r3/route_$i.log 2>&1 || { tail -3 gpurun_out/r3/route_$i.log; exit 1; }
  echo "16k $1=$2 $(grep -h '^{' gpurun_out/r3/route_$i.log | grep -o '"value": [0-9.]*\|"manager_ms": {[^}]*}' | tr '\n' ' ')" >> $out
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/t16r -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/r3/t16r.log 2>&1
cat $out
