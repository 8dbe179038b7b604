#!/bin/bash
# Validation of the current tree: GPU suite, smoke, 2-rank shared-GPU run,
# configs 2 and 3
set -o pipefail
mkdir -p gpurun_out/v
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest --maxfail=6 -v --timeout 150 --timeout-method thread -m gpu tests/ > gpurun_out/v/suite.log 2>&1
rc0=$?
tail -3 gpurun_out/v/suite.log; grep -E "FAILED|ERROR" gpurun_out/v/suite.log | head -10
[ $rc0 -le 1 ] &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1 &&
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29581 \
   bench.py --gpus 2 --size 16384 --nb 512 --steps 3 --warmup 1 --share-gpu --cores 3 > gpurun_out/v/m2.log 2>&1 &&
timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 5 --warmup 1 > gpurun_out/v/b16.log 2>&1 &&
timeout -k 10 240 python3 bench.py --steps 5 --warmup 1 > gpurun_out/v/b64.log 2>&1
rc=$?
tail -1 gpurun_out/v/smoke.log; grep -h '^{' gpurun_out/v/m2.log gpurun_out/v/b16.log gpurun_out/v/b64.log | cut -c1-220
exit $((rc0 + rc))
