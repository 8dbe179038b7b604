#!/bin/bash
# 8-rank P4xQ2 shared-GPU check, repeated, with and without extra critical streams
set -o pipefail
mkdir -p gpurun_out
for x in 7 0 7; do
PARSEC_MCA_device_hip_critical_streams=$x timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 2954$x \
    bench.py --gpus 8 --size 8192 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 1 > gpurun_out/multi8s_$x.log 2>&1 || exit 1
echo "xcrit=$x $(grep -o '"max_rel_error_vs_torch_cholesky": [0-9.e+-]*' gpurun_out/multi8s_$x.log)"
done
for n in 2 4; do
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2956$n \
    bench.py --gpus $n --size 8192 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 2 > gpurun_out/multi${n}s.log 2>&1 || exit 1
echo "n=$n $(grep -o '"max_rel_error_vs_torch_cholesky": [0-9.e+-]*' gpurun_out/multi${n}s.log)"
done
