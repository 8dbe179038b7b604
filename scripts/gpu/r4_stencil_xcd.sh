#!/bin/bash
# Config 5 (DTD 3D stencil 1024^3, 256^3 blocks, 1 GPU): XCD-contiguous workgroup
# remap of the stencil kernel (PARSEC_STENCIL_XCD) A/B + kernel stats of each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stx
timeout -k 10 200 python3 -u -m pytest tests -m gpu -x -q -k stencil --timeout 120 --timeout-method thread > gpurun_out/stx/tests.log 2>&1 || { tail -30 gpurun_out/stx/tests.log; exit 1; }
tail -1 gpurun_out/stx/tests.log
for spec in "x1;PARSEC_STENCIL_XCD=1" "x0;PARSEC_STENCIL_XCD=0" "x1b;PARSEC_STENCIL_XCD=1" "x0b;PARSEC_STENCIL_XCD=0"; do
  IFS=';' read -r name envs <<< "$spec"
  env $envs timeout -k 10 200 python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 20 > gpurun_out/stx/$name.json 2> gpurun_out/stx/$name.err || { tail -5 gpurun_out/stx/$name.err; exit 1; }
  echo "$name $envs $(cut -c1-110 gpurun_out/stx/$name.json)"
done
for x in 1 0; do
  PARSEC_STENCIL_XCD=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stx/p$x -o run -- python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 20 > gpurun_out/stx/p$x.log 2>&1 || { tail -5 gpurun_out/stx/p$x.log; exit 1; }
  f=$(find gpurun_out/stx/p$x -name "*kernel_stats.csv" -print -quit); cp $f gpurun_out/stx/kstats_x$x.csv; rm -rf gpurun_out/stx/p$x
  echo "xcd=$x"; head -4 gpurun_out/stx/kstats_x$x.csv | cut -c1-160
done
