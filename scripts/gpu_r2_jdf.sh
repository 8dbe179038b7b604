#!/bin/bash
# GPU suite (incl. split-K and JDF DPOTRF tests) + A/B: IR vs ptgpp-compiled JDF taskpool,
# split-K tail off/on, at the config-2 and headline sizes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/j_tests.log 2>&1; trc=$?
tail -n 3 gpurun_out/j_tests.log
[ $trc -ge 124 ] && exit $trc
timeout -k 10 240 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/j_16k_ir.log 2>&1 && \
timeout -k 10 240 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 --taskpool jdf > gpurun_out/j_16k_jdf.log 2>&1 && \
timeout -k 10 240 env PARSEC_GEMM_SPLITK=1 python bench.py --gpus 1 --size 16384 --nb 512 --steps 5 --warmup 2 > gpurun_out/j_16k_splitk.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/j_64k_ir.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 3 --warmup 1 --taskpool jdf > gpurun_out/j_64k_jdf.log 2>&1 && \
timeout -k 10 300 env PARSEC_GEMM_SPLITK=1 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/j_64k_splitk.log 2>&1
rc=$?
for f in gpurun_out/j_16k_ir.log gpurun_out/j_16k_jdf.log gpurun_out/j_16k_splitk.log gpurun_out/j_64k_ir.log gpurun_out/j_64k_jdf.log gpurun_out/j_64k_splitk.log; do
  echo "$f $(grep -h '"metric"' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("residual"))' 2>/dev/null)"
done
exit $(( trc > rc ? trc : rc ))
