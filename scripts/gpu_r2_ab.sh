#!/bin/bash
# Interleaved A/B of DPOTRF bench variants (env settings), 16k/nb512 and 64k/nb1024.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.log
run() {  # tag size nb steps warmup env...
  local tag=$1 n=$2 nb=$3 st=$4 wu=$5; shift 5
  timeout -k 10 300 env "$@" python bench.py --gpus 1 --size $n --nb $nb --steps $st --warmup $wu > gpurun_out/ab_$tag.log 2>&1 || return $?
  echo "$tag $(grep -h '"metric"' gpurun_out/ab_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/ab.log
}
for rep in 1 2; do
  run base16_$rep 16384 512 6 2 PARSEC_GEMM_CHUNK_FILL=0 PARSEC_GEMM_SPLITK=0 || exit $?
  run fill16_$rep 16384 512 6 2 PARSEC_GEMM_CHUNK_FILL=1 PARSEC_GEMM_SPLITK=0 || exit $?
  run fillsk16_$rep 16384 512 6 2 PARSEC_GEMM_CHUNK_FILL=1 PARSEC_GEMM_SPLITK=1 || exit $?
  run sk16_$rep 16384 512 6 2 PARSEC_GEMM_CHUNK_FILL=0 PARSEC_GEMM_SPLITK=1 || exit $?
done
run base64 65536 1024 3 1 PARSEC_GEMM_CHUNK_FILL=0 PARSEC_GEMM_SPLITK=0 || exit $?
run fill64 65536 1024 3 1 PARSEC_GEMM_CHUNK_FILL=1 PARSEC_GEMM_SPLITK=0 || exit $?
run fillsk64 65536 1024 3 1 PARSEC_GEMM_CHUNK_FILL=1 PARSEC_GEMM_SPLITK=1 || exit $?
cat gpurun_out/ab.log
