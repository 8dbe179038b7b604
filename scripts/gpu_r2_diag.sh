#!/bin/bash
# 4 independent single-rank DPOTRF processes on one GPU; host LAPACK reference, torch GPU cholesky compared too
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 0 1 2 3; do env REPEAT=3 CHECK_TORCH_GPU=1 timeout -k 5 150 python tests/mp/gpu_dist.py dpotrf 0 1 tr_${r}_$$ 8192 512 1 1 > gpurun_out/tr_$r.log 2>&1 & done
wait
for r in 0 1 2 3; do echo "== $r"; grep -h "bad_reps\|bad tiles\|torch GPU" gpurun_out/tr_$r.log | cut -c1-160; done
for r in 0 1; do env REPEAT=3 CHECK_TORCH_GPU=1 timeout -k 5 150 python tests/mp/gpu_dist.py dpotrf $r 2 ipc_$$ 8192 512 2 1 > gpurun_out/ip_$r.log 2>&1 & done
wait
for r in 0 1; do echo "== ipc $r"; grep -h "bad_reps\|bad tiles\|torch GPU" gpurun_out/ip_$r.log | cut -c1-160; done
