#!/bin/bash
# CE GPU test, tile-POTRF phase stamps, and a kernel trace of config 2 reduced to
# the per-panel critical chain.
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_multirank_gpu.py -k comm_engine > gpurun_out/r3/ce.log 2>&1 &&
PARSEC_POTRF_STAMPS=1 timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/r3/kstamps.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/t16 -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/r3/t16.log 2>&1
rc=$?; tail -3 gpurun_out/r3/ce.log; cat gpurun_out/r3/kstamps.log; grep -h '^{' gpurun_out/r3/t16.log | cut -c1-200
f=$(find gpurun_out/r3/t16 -name "*kernel_trace.csv" -print -quit); [ -n "$f" ] && python3 scripts/critical_chain.py $f 512 16384 > gpurun_out/r3/chain16.txt; cat gpurun_out/r3/chain16.txt
exit $rc
