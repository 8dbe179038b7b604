#!/bin/bash
# Which change broke the 4-rank GPU DTD stencil? One run per suspect.
mkdir -p gpurun_out
: > gpurun_out/sb.log
for v in "X=1" "PARSEC_MEMCPY_LEGACY=1" "PARSEC_MCA_ptg_dep_management=dynamic-hash-table" "PARSEC_GEMM_SPLITK=0 PARSEC_GEMM_CHUNK_FILL=0"; do
  timeout -k 10 200 env $v python -u -m pytest tests/test_multirank_gpu.py -x -q -k stencil --timeout 150 --timeout-method thread > gpurun_out/sb_tmp.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -h 'err' gpurun_out/sb_tmp.log | head -4 | tr '\n' ' ')" >> gpurun_out/sb.log
  [ $rc -ge 124 ] && break
done
cat gpurun_out/sb.log
