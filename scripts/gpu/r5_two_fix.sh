#!/bin/bash
# Two logical devices + capped cache after pinning GPU transfer sources: repeated runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/twofix; mkdir -p $O
i=0; bad=0
for spec in "1 256 0.3" "1 256 0.3" "1 256 0.3" "1 512 0.3" "1 512 0.3" "0 256 0.3" "1 256 0.2" "1 128 0.3"; do
  set -- $spec; i=$((i+1))
  PARSEC_MCA_device_hip_peer_stage_in=$1 timeout -k 10 150 python3 tests/mp/gpu_two_devices.py 4096 $2 $3 > $O/r_$i.log 2>&1; rc=$?
  echo "peer=$1 nb=$2 cache=$3 rc=$rc $(grep two_devices $O/r_$i.log | cut -c1-260)"
  if [ $rc -ge 124 ]; then exit 1; fi
  [ $rc -ne 0 ] && bad=$((bad+1))
done
echo "bad=$bad"
