#!/bin/bash
# Round 6: LDS bank conflicts per kernel (one PMC pass each, kernel trace only): DGEQRF 8k and DPOTRF 8k.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ldspmc; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/q -o run -- python3 benchmarks/bench_workloads.py qr --size 8192 --nb 512 --steps 1 --warmup 0 > $O/q.log 2>&1 || { tail -5 $O/q.log; exit 1; }
f=$(find $O/q -name "*counter_collection.csv" -print -quit); python3 scripts/lds_conflicts.py $f > $O/qr_lds.txt; cat $O/qr_lds.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $O/p -o run -- python3 bench.py --size 8192 --nb 512 --steps 1 --warmup 0 > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
f=$(find $O/p -name "*counter_collection.csv" -print -quit); python3 scripts/lds_conflicts.py $f > $O/potrf_lds.txt; cat $O/potrf_lds.txt
rm -rf $O/q $O/p
