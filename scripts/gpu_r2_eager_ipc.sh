#!/bin/bash
# Eager IPC descriptors in activations: multi-rank GPU tests, then A/B on shared-GPU rank runs
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/mr_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/mr_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
R2="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
R4="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
for e in 1 0; do
  PARSEC_MCA_comm_eager_ipc=$e timeout -k 10 120 $R2 --master-port 2961$e bench.py --gpus 2 --size 16384 --nb 1024 --steps 3 --warmup 1 --share-gpu --cores 2 --check > gpurun_out/e${e}_s2.log 2>&1 || exit $?
  echo "eager=$e 2r $(grep -h '^{' gpurun_out/e${e}_s2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("max_rel_error_vs_torch_cholesky"))')"
  PARSEC_MCA_comm_eager_ipc=$e timeout -k 10 120 $R4 --master-port 2962$e bench.py --gpus 4 --size 4096 --nb 1024 --steps 2 --warmup 1 --share-gpu --cores 2 --check > gpurun_out/e${e}_s4.log 2>&1 || exit $?
  echo "eager=$e 4r $(grep -h '^{' gpurun_out/e${e}_s4.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("max_rel_error_vs_torch_cholesky"))')"
done
