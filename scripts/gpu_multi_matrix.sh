#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
i=0
for cfg in "4 1" "4 1" "8 2" "8 2" "2 1" "2 1" "8 1 device_hip_max_streams 1" "8 1 device_hip_max_streams 1"; do
set -- $cfg
n=$1; c=$2; extra=""
[ -n "$3" ] && extra="--mca $3 $4"
i=$((i+1))
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 296$((10+i)) \
    bench.py --gpus $n --size 8192 --nb 512 --steps 2 --warmup 1 --share-gpu --check --cores $c $extra > gpurun_out/mm_$i.log 2>&1 || { tail -5 gpurun_out/mm_$i.log; exit 1; }
echo "n=$n cores=$c $extra: $(grep -o '"max_rel_error_vs_torch_cholesky": [0-9.e+-]*' gpurun_out/mm_$i.log)"
done
