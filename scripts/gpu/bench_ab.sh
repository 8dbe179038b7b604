#!/bin/bash
# Generic bench.py A/B on the GPU box. Each argument is "name;ENV=VAL ...;bench args";
# rows go to gpurun_out/ab/<tag>.txt (tag = $AB_TAG or "ab"). Example:
#   bash scripts/gpu/bench_ab.sh "g2;;--size 16384 --nb 512 --mca device_hip_group_rounds 2" \
#                                "g0;;--size 16384 --nb 512 --mca device_hip_group_rounds 0"
set -o pipefail
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/ab/${AB_TAG:-ab}.txt; : > $out
for spec in "$@"; do
  IFS=';' read -r name envs args <<< "$spec"
  env X_AB=1 $envs timeout -k 10 300 python3 bench.py $args > gpurun_out/ab/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/ab/$name.log; exit 1; }
  echo "$name [$envs] $args : $(grep -h '^{' gpurun_out/ab/$name.log | cut -c90-150)" >> $out
done
cat $out
