#!/bin/bash
# Round 5: where a tile POTRF's time goes under load (config 2): step kernels
# running vs the gaps between their launches (rocprofv3 kernel trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ptrace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t16 -o run -- python3 bench.py --size 16384 --nb 512 --steps 1 --warmup 1 > $O/t16.log 2>&1 || { tail -5 $O/t16.log; exit 1; }
t=$(find $O/t16 -name "*kernel_trace.csv" -print -quit)
python3 scripts/potrf_gaps.py $t 512 16384 > $O/gaps16.txt 2>&1; cat $O/gaps16.txt
python3 scripts/critical_chain.py $t 512 16384 > $O/chain16.txt 2>&1; tail -3 $O/chain16.txt
rm -rf $O/t16
