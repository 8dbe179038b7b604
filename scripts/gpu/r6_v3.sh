#!/bin/bash
# Round 6: copy-stream load (engine-timed copy spans) and 256x128 GEMM tiles.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6copy; mkdir -p $O
for spec in "evict;16384 512 0.25" "fit;16384 512 2.0" "two;16384 512 0.0 2" "evict1k;16384 1024 0.25"; do
  IFS=';' read -r name args <<< "$spec"
  timeout -k 10 200 python3 scripts/copy_stream_profile.py $args > $O/$name.txt 2>&1 || { echo "$name failed"; tail -5 $O/$name.txt; exit 1; }
  tail -1 $O/$name.txt
done
O=gpurun_out/r6gemm; mkdir -p $O
for v in 0 13 14; do
  PARSEC_GEMM_PAD_TEST=1 PARSEC_GEMM_VARIANT=$v timeout -k 10 200 python3 scripts/kbench_gemm.py > $O/k$v.txt 2>&1 || { echo "kbench $v failed"; tail -5 $O/k$v.txt; exit 1; }
  cat $O/k$v.txt
done
AB_TAG=r6_gemm bash scripts/gpu/bench_ab.sh "c3v0;;--steps 3 --warmup 1" "c3v13;PARSEC_GEMM_VARIANT=13;--steps 3 --warmup 1" "c3v14;PARSEC_GEMM_VARIANT=14;--steps 3 --warmup 1" "c3v0b;;--steps 3 --warmup 1" || exit 1
