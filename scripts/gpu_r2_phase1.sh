#!/bin/bash
# Round 2: full GPU test suite, then the 1-GPU benches (residual checked) and a kernel profile of config 2.
set -o pipefail
mkdir -p gpurun_out/prof16k
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/p1_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/p1_bench16k.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/p1_bench64k.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16k -o run -- python bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/p1_prof16k.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/p1_tests.log | tail -2
for f in gpurun_out/p1_bench*.log gpurun_out/p1_prof16k.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -n 2 | cut -c1-400; done
find gpurun_out/prof16k -name "*kernel_stats.csv" | head -2
exit $rc
