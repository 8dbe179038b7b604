#!/bin/bash
# Wave-priority A/B (s_setprio on the critical stream's kernels), config 2 and 3
set -o pipefail
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r3/prio_ab.txt; : > $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/r3/kt.log 2>&1 || { tail -5 gpurun_out/r3/kt.log; exit 1; }
for w in 1 0; do
  timeout -k 10 200 python3 bench.py --size 16384 --nb 512 --steps 3 --warmup 1 --mca device_hip_wave_priority $w > gpurun_out/r3/prio16_$w.log 2>&1 || exit 1
  echo "16k wave_priority=$w $(grep -h '^{' gpurun_out/r3/prio16_$w.log | cut -c90-140)" >> $out
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/t16p -o run -- python3 bench.py --gpus 1 --size 16384 --nb 512 --steps 2 --warmup 1 > gpurun_out/r3/t16p.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > gpurun_out/r3/prio64_1.log 2>&1 || exit 1
echo "64k wave_priority=1 $(grep -h '^{' gpurun_out/r3/prio64_1.log | cut -c90-140)" >> $out
cat $out
