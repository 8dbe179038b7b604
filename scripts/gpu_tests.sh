#!/bin/bash
# GPU test run with per-test progress and a per-test timeout, then the
# 2-rank shared-GPU validation of the distributed path.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|Timeout|passed|failed" gpurun_out/pytest_gpu.log | tail -n 40 | cut -c1-250
if [ $rc -eq 0 ]; then
  PARSEC_BENCH_VERBOSE=1 PARSEC_MCA_debug_verbose=10 timeout -k 10 60 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --size 2048 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 3 \
      > gpurun_out/multi2s.log 2>&1
  rc=$?
  echo "== multi2s rc=$rc"; grep -v "amdgpu.ids\|socket.cpp\|comm\]" gpurun_out/multi2s.log | tail -n 16 | cut -c1-250
fi
exit $rc
