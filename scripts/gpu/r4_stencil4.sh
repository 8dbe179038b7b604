#!/bin/bash
# DTD 3D stencil, 1 rank and 4 ranks sharing the box's GPU (halo faces cross
# ranks over IPC and stay in HBM): Gpoint/s lines for profiles/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/st4
timeout -k 10 200 python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 20 > gpurun_out/st4/r1.json 2> gpurun_out/st4/r1.err || { tail -5 gpurun_out/st4/r1.err; exit 1; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 benchmarks/bench_workloads.py stencil --share-gpu --size 1024 --b 256 --iters 20 > gpurun_out/st4/r4.json 2> gpurun_out/st4/r4.err || { tail -20 gpurun_out/st4/r4.err; exit 1; }
cat gpurun_out/st4/r1.json gpurun_out/st4/r4.json
