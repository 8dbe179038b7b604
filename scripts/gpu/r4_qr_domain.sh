#!/bin/bash
# DGEQRF config 4: hierarchical tree domain size A/B at 32k (flat = 0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qrd
ENVS=${ENVS:-PARSEC_QR_DUMMY=0}
for dom in 0 16 32; do
  env $ENVS timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 --qr-domain $dom > gpurun_out/qrd/d${dom}${TAG}.json 2> gpurun_out/qrd/d${dom}${TAG}.err || { tail -5 gpurun_out/qrd/d${dom}${TAG}.err; exit 1; }
  echo "domain $dom $ENVS $(cut -c1-120 gpurun_out/qrd/d${dom}${TAG}.json)"
done
