#!/bin/bash
# Stream routing A/B after the bulk-group split: hp (non-critical) tasks on the
# critical stream (1) or on the bulk streams (0), bulk group size and in-flight depth
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3/route_ab2.txt; : > $out
i=0
for cfg in "1 2 2" "0 2 2" "0 1 1" "0 2 1" "1 1 2" "1 2 1" "1 2 2"; do
  set -- $cfg; i=$((i+1))
  timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 4 --warmup 1 --mca device_hip_hp_on_critical_stream $1 --mca device_hip_group_rounds $2 --mca device_hip_max_inflight_batches $3 > gpurun_out/r3/rt$i.log 2>&1 || exit 1
  echo "16k hp_on_crit=$1 group_rounds=$2 max_inflight=$3 $(grep -h '^{' gpurun_out/r3/rt$i.log | cut -c90-140)" >> $out
done
cat $out
W="python3 benchmarks/bench_workloads.py qr"
for cfg in "16384 32 0" "16384 64 0" "16384 16 0" "16384 32 4" "16384 64 4" "32768 64 0"; do
  set -- $cfg
  timeout -k 10 300 $W --n $1 --nb 512 --ib $2 --qr-domain $3 --steps 1 --check > gpurun_out/r3/q_$1_$2_$3.log 2>&1 || exit 1
  echo "qr n=$1 ib=$2 domain=$3 $(grep -h '^{' gpurun_out/r3/q_$1_$2_$3.log | cut -c50-120) $(grep -ho 'residual[^,]*' gpurun_out/r3/q_$1_$2_$3.log | tail -1)" >> $out
done
cat $out
