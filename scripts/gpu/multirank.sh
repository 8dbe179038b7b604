#!/bin/bash
# GPU suite + smoke, per-edge comm latency of 2 shared-GPU ranks (config 2
# shape, eager IPC off / on), and the exact headline config on 8 ranks
# (N=65536, nb=1024, P4xQ2) sharing the box's one GPU.
set -o pipefail
mkdir -p gpurun_out/m
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest --maxfail=6 -v --timeout 150 --timeout-method thread -m gpu tests/ > gpurun_out/m/suite.log 2>&1
rc0=$?
tail -3 gpurun_out/m/suite.log; grep -E "FAILED|ERROR" gpurun_out/m/suite.log | head -10
[ $rc0 -le 1 ] &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/m/smoke.log 2>&1 &&
for e in 0 1; do
  PARSEC_MCA_profile_filename=$GRAFT_REPO_ROOT/gpurun_out/m/e$e PARSEC_MCA_comm_eager_ipc=$e timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2955$e \
     bench.py --gpus 2 --size 16384 --nb 512 --steps 2 --warmup 1 --share-gpu --cores 3 > gpurun_out/m/e$e.log 2>&1 || exit 1
  python3 scripts/comm_edges.py gpurun_out/m/e$e 2 > gpurun_out/m/edges_e$e.txt 2>&1
done &&
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29561 \
   bench.py --gpus 8 --steps 1 --warmup 1 --share-gpu --cores 1 --mca device_hip_memory_max 17179869184 > gpurun_out/m/h8.log 2>&1
rc=$?
tail -2 gpurun_out/m/smoke.log; grep -h '^{' gpurun_out/m/e0.log gpurun_out/m/e1.log gpurun_out/m/h8.log | cut -c1-330; cat gpurun_out/m/edges_e*.txt
rm -f gpurun_out/m/*.prof
exit $((rc0 + rc))
