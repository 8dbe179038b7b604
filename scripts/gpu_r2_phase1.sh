#!/bin/bash
# Round 2 phase 1: new headline/multi-rank GPU tests, then the 1-GPU benches (residual checked).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_headline_gpu.py tests/test_multirank_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/p1_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/p1_bench16k.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/p1_bench64k.log 2>&1
rc=$?
for f in gpurun_out/p1_*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -n 25 | cut -c1-300; done
exit $rc
