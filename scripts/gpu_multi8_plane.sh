#!/bin/bash
# 8-rank P4xQ2 shared-GPU check: IPC vs host-staged device data plane, 3 runs each
set -o pipefail
mkdir -p gpurun_out
i=0
for plane in ipc host ipc host ipc host; do
i=$((i+1))
PARSEC_MCA_comm_device_plane=$plane timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 295$((50+i)) \
    bench.py --gpus 8 --size 8192 --nb 512 --steps 2 --warmup 1 --share-gpu --check --cores 1 > gpurun_out/m8_$plane$i.log 2>&1 || { tail -5 gpurun_out/m8_$plane$i.log; exit 1; }
echo "$plane run $i: $(grep -o '"max_rel_error_vs_torch_cholesky": [0-9.e+-]*' gpurun_out/m8_$plane$i.log)"
done
