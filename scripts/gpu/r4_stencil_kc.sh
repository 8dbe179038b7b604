#!/bin/bash
# Config 5: stencil kernel planes per workgroup (PARSEC_STENCIL_KC) and 4x unrolled k loop
# (PARSEC_STENCIL_UNR) A/B, XCD remap on.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stk
timeout -k 10 200 python3 -u -m pytest tests -m gpu -x -q -k stencil --timeout 120 --timeout-method thread > gpurun_out/stk/tests.log 2>&1 || { tail -30 gpurun_out/stk/tests.log; exit 1; }
PARSEC_STENCIL_UNR=4 PARSEC_STENCIL_KC=64 timeout -k 10 200 python3 -u -m pytest tests -m gpu -x -q -k stencil --timeout 120 --timeout-method thread >> gpurun_out/stk/tests.log 2>&1 || { tail -30 gpurun_out/stk/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/stk/tests.log
for spec in "kc32;" "kc64;PARSEC_STENCIL_KC=64" "kc16;PARSEC_STENCIL_KC=16" "kc128;PARSEC_STENCIL_KC=128" "u4;PARSEC_STENCIL_UNR=4" "kc64u4;PARSEC_STENCIL_KC=64 PARSEC_STENCIL_UNR=4" \
            "kc32b;" "kc64b;PARSEC_STENCIL_KC=64" "u4b;PARSEC_STENCIL_UNR=4" "kc64u4b;PARSEC_STENCIL_KC=64 PARSEC_STENCIL_UNR=4"; do
  IFS=';' read -r name envs <<< "$spec"
  env X_AB=1 $envs timeout -k 10 200 python3 benchmarks/bench_workloads.py stencil --size 1024 --b 256 --iters 20 > gpurun_out/stk/$name.json 2> gpurun_out/stk/$name.err || { tail -5 gpurun_out/stk/$name.err; exit 1; }
  echo "$name [$envs] $(cut -c1-100 gpurun_out/stk/$name.json)"
done
