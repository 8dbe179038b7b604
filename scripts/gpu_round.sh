#!/bin/bash
# One GPU session: smoke, GPU tests, benches. Every GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/bench_16k.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench_64k.log 2>&1
rc=$?
tail -5 gpurun_out/*.log
exit $rc
