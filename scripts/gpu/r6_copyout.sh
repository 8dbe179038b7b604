#!/bin/bash
# Round 6: device-to-host write-back / W2R on a copy stream of their own (device_hip_copy_out_stream) in the out-of-core DPOTRF.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/cout; mkdir -p $O
export GPU_MAX_HW_QUEUES=8
PARSEC_MCA_device_hip_copy_out_stream=1 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_memory.py tests/test_dpotrf_gpu.py > $O/t.log 2>&1 || { grep -E "FAILED|Error" $O/t.log | head; tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
: > $O/ab.txt
for spec in "b;0;16384 512 0.25" "s;1;16384 512 0.25" "b1k;0;16384 1024 0.25" "s1k;1;16384 1024 0.25" "b2;0;16384 512 0.25" "s2;1;16384 512 0.25" "b1k2;0;16384 1024 0.25" "s1k2;1;16384 1024 0.25"; do
  IFS=';' read -r name on args <<< "$spec"
  PARSEC_MCA_device_hip_copy_out_stream=$on timeout -k 10 200 python3 scripts/copy_stream_profile.py $args > $O/$name.txt 2>&1 || { echo "$name failed"; tail -5 $O/$name.txt; exit 1; }
  echo "$name copy_out_stream=$on $(tail -1 $O/$name.txt | cut -c1-160)" >> $O/ab.txt
done
cat $O/ab.txt
