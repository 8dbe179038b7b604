#!/bin/bash
# Round 6: batched TSMQR apply rates and the split between its three grouped GEMM launches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/qra6; mkdir -p $O
timeout -k 10 200 python3 scripts/kbench_qr_apply.py > $O/k.log 2>&1 || { tail -5 $O/k.log; exit 1; }
cat $O/k.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 scripts/kbench_qr_apply.py > $O/kp.log 2>&1 || { tail -5 $O/kp.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" -print -quit); cp $f $O/stats.csv; cut -c1-180 $O/stats.csv | head -8; rm -rf $O/p
