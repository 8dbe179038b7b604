#!/bin/bash
# tests, benches and a kernel profile; each GPU step time-limited, chain stops on failure
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/bench_16k.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 3 --warmup 1 --check > gpurun_out/bench_16k_check.log 2>&1 && \
PARSEC_GEMM_TILE=64 timeout -k 10 300 python bench.py --gpus 1 --n 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/bench_16k_t64.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/bench_64k.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/p16k -o run -- python3 bench.py --gpus 1 --n 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/prof/bench16k.log 2>&1
rc=$?
for f in gpurun_out/pytest_gpu.log gpurun_out/bench_*.log; do echo "== $f"; tail -n 3 $f | cut -c1-400; done
exit $rc
