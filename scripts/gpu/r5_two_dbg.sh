#!/bin/bash
# Two logical devices + capped tile cache: which combination breaks the factor.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/twodbg; mkdir -p $O
for spec in "1 256 0.3" "0 256 0.3" "1 512 0.3" "0 512 0.3" "1 256 0.0" "0 256 0.0" "1 256 0.6" "0 256 0.6"; do
  set -- $spec
  PARSEC_MCA_device_hip_peer_stage_in=$1 timeout -k 10 150 python3 tests/mp/gpu_two_devices.py 4096 $2 $3 > $O/r_$1_$2_$3.log 2>&1; rc=$?
  echo "peer=$1 nb=$2 cache=$3 rc=$rc $(grep two_devices $O/r_$1_$2_$3.log | cut -c1-260)"
  if [ $rc -ge 124 ]; then exit 1; fi
done
