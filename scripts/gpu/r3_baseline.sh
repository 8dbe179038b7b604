#!/bin/bash
# Round-3 baseline: critical-path kernel latencies, config 2 (both taskpools), kernel trace of config 2
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 scripts/kbench_critical.py > gpurun_out/r3/kcrit.log 2>&1 &&
timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/r3/b16_ir.log 2>&1 &&
timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 --taskpool jdf > gpurun_out/r3/b16_jdf.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/p16 -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/r3/p16.log 2>&1
rc=$?; cat gpurun_out/r3/kcrit.log; grep -h '^{' gpurun_out/r3/*.log | cut -c1-300; exit $rc
