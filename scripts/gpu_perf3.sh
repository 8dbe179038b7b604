#!/bin/bash
# GEMM kernel check + DPOTRF benches + kernel profile of the 16k config.
set -o pipefail
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_kern.log 2>&1 && \
for v in 0 1; do PARSEC_GEMM_VARIANT=$v timeout -k 10 120 python scripts/kbench_gemm.py >> gpurun_out/gemm_variants.log 2>&1 || exit $?; done && \
timeout -k 10 300 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/bench_16k.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/bench_64k.log 2>&1 && \
PARSEC_GEMM_VARIANT=1 timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/bench_64k_v1.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/p64k -o run -- python3 bench.py --gpus 1 --steps 1 --warmup 1 > gpurun_out/prof/bench64k.log 2>&1
rc=$?
tail -n 2 gpurun_out/pytest_kern.log; grep -v amdgpu.ids gpurun_out/gemm_variants.log
for f in gpurun_out/bench_*.log gpurun_out/prof/bench64k.log; do echo "== $f"; grep "^{" $f | cut -c1-330; done
exit $rc
