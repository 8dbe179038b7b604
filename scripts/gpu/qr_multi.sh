#!/bin/bash
# DGEQRF: 8 ranks on the P4xQ2 grid sharing the box's GPU (config 4's process
# grid, R checked over all ranks), then the TS-domain sweep at 32k on one GPU
set -o pipefail
mkdir -p gpurun_out/qm
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/qm/qr.txt; : > $out
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 \
   benchmarks/bench_workloads.py qr --size 16384 --nb 512 --steps 1 --warmup 1 --cores 1 --share-gpu --check > gpurun_out/qm/q8.log 2>&1 || { tail -20 gpurun_out/qm/q8.log; exit 1; }
grep -h '^{' gpurun_out/qm/q8.log | cut -c1-400 >> $out
for d in 0 8 16; do
  timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --n 32768 --nb 512 --steps 1 --warmup 1 --qr-domain $d --check > gpurun_out/qm/q32_$d.log 2>&1 || exit 1
  grep -h '^{' gpurun_out/qm/q32_$d.log | cut -c1-400 >> $out
done
cat $out
