#!/bin/bash
# Split-K tail of the 128x128 grouped DGEMM: correctness, full GPU suite after the
# PTG dependency-mode changes, and A/B of the DPOTRF benches (PARSEC_GEMM_SPLITK).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/s_tests.log 2>&1 && \
timeout -k 10 240 env PARSEC_GEMM_SPLITK=0 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/s_16k_off.log 2>&1 && \
timeout -k 10 240 env PARSEC_GEMM_SPLITK=1 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/s_16k_on.log 2>&1 && \
timeout -k 10 300 env PARSEC_GEMM_SPLITK=0 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/s_64k_off.log 2>&1 && \
timeout -k 10 300 env PARSEC_GEMM_SPLITK=1 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/s_64k_on.log 2>&1
rc=$?
tail -3 gpurun_out/s_tests.log
grep -h '"metric"' gpurun_out/s_16k_off.log gpurun_out/s_16k_on.log gpurun_out/s_64k_off.log gpurun_out/s_64k_on.log | cut -c1-200
exit $rc
