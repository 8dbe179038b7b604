#!/bin/bash
# Forced eviction at N=16384 (25 % cache), and the shared-GPU oracle probe
# (torch GPU Cholesky in 4 concurrent processes: runtime absent / imported / initialised)
set -o pipefail
mkdir -p gpurun_out/x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_memory.py > gpurun_out/x/evict.log 2>&1
rc0=$?; grep -E "PASSED|FAILED|evict N" gpurun_out/x/evict.log | cut -c1-250
[ $rc0 -le 1 ] &&
for m in none import init none; do
  echo "== mode $m" >> gpurun_out/x/oracle.log
  timeout -k 10 200 python3 scripts/oracle_probe.py --procs 4 --mode $m --n 8192 >> gpurun_out/x/oracle.log 2>&1 || exit 1
done
rc=$?; grep -v amdgpu.ids gpurun_out/x/oracle.log; exit $((rc0+rc))
