#!/bin/bash
# Bulk group size A/B (device_hip_group_rounds: 0 = one group per scheduling
# round, k = close a bulk group after k rounds of resident GEMM workgroups)
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3/group_ab.txt; : > $out
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python3 bench.py "$@" > gpurun_out/r3/grp_$n.log 2>&1 || return 1
  echo "$n $* $(grep -h '^{' gpurun_out/r3/grp_$n.log | cut -c90-140)" >> $out
}
for g in 0 1 2 4 2 1; do run 16_g${g}_$RANDOM --size 16384 --nb 512 --steps 4 --warmup 1 --mca device_hip_group_rounds $g || exit 1; done
for g in 2 0 1; do run 64_g$g --steps 2 --warmup 1 --mca device_hip_group_rounds $g || exit 1; done
PARSEC_BENCH_VERBOSE=1 timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 1 --warmup 1 --mca device_hip_trace_launches 1 > gpurun_out/r3/mgr16g.log 2> gpurun_out/r3/mgr16g.err
rc=$?
cat $out; exit $rc
