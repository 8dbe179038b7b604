#!/bin/bash
# 16-wave 256x128 / 128x256 GEMM variants vs the 8-wave default; numerics; DPOTRF benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rm -f gpurun_out/gemm_variants.log
for v in 0 9 10; do PARSEC_GEMM_VARIANT=$v timeout -k 10 120 python scripts/kbench_gemm.py >> gpurun_out/gemm_variants.log 2>&1 || exit $?; done && \
for v in 9 10; do PARSEC_GEMM_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "dgemm or trsm_through or inverse" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_v$v.log 2>&1 || exit $?; done && \
for v in 0 9 10; do PARSEC_GEMM_VARIANT=$v timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/b64k_v$v.log 2>&1 || exit $?; done
rc=$?
grep -v amdgpu gpurun_out/gemm_variants.log; tail -qn 1 gpurun_out/pytest_v*.log
for f in gpurun_out/b64k_v*.log; do echo -n "$f "; grep "^{" $f | python3 -c "import json,sys; [print(d['value'], d['ms_per_step'], d.get('gpu_kernel_launches')) for d in map(json.loads, sys.stdin)]"; done
exit $rc
