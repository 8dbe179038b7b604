#!/bin/bash
# MFMA/VALU co-issue probe, grouped-GEMM kernel variants, then GEMM numerics and a 4-rank shared-GPU DPOTRF check.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 60 tools/kbench/mfma_valu_probe > gpurun_out/mfma_valu_probe.log 2>&1 && \
for v in "0 0" "0 1" "1 1" "2 1" "3 1" "4 1"; do
  set -- $v
  PARSEC_GEMM_VARIANT=$1 PARSEC_GEMM_FULL=$2 timeout -k 10 120 python scripts/kbench_gemm.py >> gpurun_out/gemm_variants.log 2>&1 || exit $?
done && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_dpotrf_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_kern.log 2>&1 && \
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 \
    bench.py --gpus 4 --size 8192 --nb 512 --steps 1 --warmup 1 --share-gpu --check --cores 2 > gpurun_out/multi4s.log 2>&1
rc=$?
cat gpurun_out/mfma_valu_probe.log; grep -v amdgpu.ids gpurun_out/gemm_variants.log; tail -n 3 gpurun_out/pytest_kern.log
grep "^{" gpurun_out/multi4s.log | cut -c1-200; grep -o '"max_rel[^,]*' gpurun_out/multi4s.log
exit $rc
