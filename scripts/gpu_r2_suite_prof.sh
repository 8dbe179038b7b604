#!/bin/bash
# Full GPU suite, then a rocprofv3 kernel-stats profile of the 16k and 64k benches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sp_tests.log 2>&1; rc=$?
tail -n 3 gpurun_out/sp_tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof16k -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 3 --warmup 1 > gpurun_out/sp_prof16k.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof64k -o run -- python3 bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/sp_prof64k.log 2>&1
rc=$?
grep -h '"metric"' gpurun_out/sp_prof16k.log gpurun_out/sp_prof64k.log | cut -c1-160
find gpurun_out/sp_prof16k gpurun_out/sp_prof64k -name "*kernel_stats.csv" | head
exit $rc
