#!/bin/bash
# Final-engine kernel statistics: config 2 (16k / nb 512) and config 3 (64k / nb 1024), rocprofv3 --kernel-trace --stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pf
for spec in "c2;--size 16384 --nb 512 --steps 3 --warmup 1" "c3;--steps 1 --warmup 1"; do
  IFS=';' read -r name a <<< "$spec"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/$name -o run -- python3 bench.py $a > gpurun_out/pf/$name.log 2>&1 || { tail -5 gpurun_out/pf/$name.log; exit 1; }
  f=$(find gpurun_out/pf/$name -name "*kernel_stats.csv" -print -quit); cp $f gpurun_out/pf/${name}_kernel_stats.csv
  t=$(find gpurun_out/pf/$name -name "*kernel_trace.csv" -print -quit); python3 scripts/trace_summary.py $t > gpurun_out/pf/${name}_summary.txt 2>&1 || true
  rm -rf gpurun_out/pf/$name
  echo "== $name"; head -8 gpurun_out/pf/${name}_kernel_stats.csv | cut -c1-180; tail -3 gpurun_out/pf/${name}_summary.txt
done
