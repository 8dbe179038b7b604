#!/bin/bash
# Round 6: anatomy of the config-2 critical chain (what the critical queue runs between tile POTRFs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/anat; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t16 -o run -- python3 bench.py --size 16384 --nb 512 --steps 1 --warmup 1 > $O/t16.log 2>&1 || { tail -5 $O/t16.log; exit 1; }
t=$(find $O/t16 -name "*kernel_trace.csv" -print -quit)
head -1 $t > $O/header.txt
python3 scripts/chain_window.py $t 512 16384 > $O/win16.txt 2>&1; cat $O/win16.txt
python3 scripts/critical_chain.py $t 512 16384 > $O/chain16.txt 2>&1; tail -2 $O/chain16.txt
gzip -c $t > $O/t16_trace.csv.gz
rm -rf $O/t16
