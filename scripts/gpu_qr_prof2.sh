#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof/qrk
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/qrk -o run -- python3 scripts/qr_kbench.py 512 > gpurun_out/prof/qrk.log 2>&1
rc=$?
f=$(find gpurun_out/prof/qrk -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | cut -c1-160
exit $rc
