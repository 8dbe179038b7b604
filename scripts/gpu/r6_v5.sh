#!/bin/bash
# Round 6 final validation: whole GPU suite, smoke, configs 3 / 2 / 4 / 5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R6_OUT=r6v5 bash scripts/gpu/r6_v1.sh || exit 1
O=gpurun_out/r6v5
timeout -k 10 300 python3 benchmarks/bench_workloads.py stencil --n 1024 --b 256 --iters 20 > $O/st.log 2>&1 || { tail -5 $O/st.log; exit 1; }
grep -h '^{' $O/st.log | cut -c1-220
timeout -k 10 300 python3 benchmarks/bench_workloads.py qr --size 32768 --nb 512 --steps 2 --warmup 1 --check > $O/qr.log 2>&1 || { tail -5 $O/qr.log; exit 1; }
grep -h '^{' $O/qr.log | cut -c1-220
